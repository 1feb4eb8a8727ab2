#!/bin/bash
# Same-box comparison: the capture-rate probe, then the DLRM bench's async
# capture at 16 / 32 threads (no overlap) and the HBM freeze.
set -o pipefail
O=${OUT:-gpurun_out/r6/uvmcap4}
mkdir -p $O
export PYTHONUNBUFFERED=1 HSBENCH_DIR=$PWD/bench_tmp
mkdir -p $HSBENCH_DIR
timeout -k 10 300 python scripts/probes/uvm_capture_probe.py --gb 8 > $O/probe.json 2> $O/probe.err || { tail -20 $O/probe.err; exit 1; }
cat $O/probe.json
for mode in "uvm_capture_threads=16" "uvm_capture_threads=32" "uvm_async_capture=False"; do
  tag=$(echo $mode | tr ' =' '_-')
  timeout -k 10 300 python scripts/probes/with_tuning.py $mode -- benchmarks/dlrm_uvm/main.py --total-gb 8 --uvm --sync-repeats 3 > $O/$tag.json 2> $O/$tag.err || { tail -20 $O/$tag.err; exit 1; }
  echo "$mode: $(tail -1 $O/$tag.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ("sync_GBps_each","freeze_gpu_ms","async_total_s","async_GBps","uvm_capture_stats","uvm_pages_per_numa_node")})')"
done
