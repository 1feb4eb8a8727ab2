#!/bin/bash
# Round 6: DLRM 8 GB UVM sync-save spread.  Each run makes
# 6 timed sync takes with their phase split, page-cache state, page faults,
# the managed pages' NUMA nodes and the writers' CPUs; runs alternate the
# process binding to the GPU's NUMA node (HIPSNAPSHOT_NUMA_BIND) off / on.
set -o pipefail
O=${OUT:-gpurun_out/r6/dlrm_var}
mkdir -p $O
export PYTHONUNBUFFERED=1 HSBENCH_DIR=$PWD/bench_tmp
mkdir -p $HSBENCH_DIR
for i in $(seq 1 ${RUNS:-2}); do
  for b in ${BINDS:-0 1}; do
    if [ $b = 1 ]; then export HIPSNAPSHOT_NUMA_BIND=1; else unset HIPSNAPSHOT_NUMA_BIND; fi
    timeout -k 10 300 python benchmarks/dlrm_uvm/main.py --total-gb 8 --uvm --sync-repeats 6 \
        > $O/bind${b}_$i.json 2> $O/bind${b}_$i.err || { tail -20 $O/bind${b}_$i.err; exit 1; }
    echo "bind=$b run $i: $(tail -1 $O/bind${b}_$i.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["sync_GBps_each"], d["uvm_pages_per_numa_node"], d["writer_cpu_nodes"], d["async_GBps"], d["freeze_gpu_ms"], d["restore_GBps"], [(x["cpu_s"], {n: (v.get("copy_GBps_1thread"), v.get("MemFree")) for n, v in x["nodes_before"].items()}) for x in d["sync_each"]][:3])')"
  done
done
