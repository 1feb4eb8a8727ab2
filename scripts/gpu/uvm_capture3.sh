#!/bin/bash
# The config-4 share (12.5 GB UVM tables, one snapshot path) and DLRM 8 GB:
# async capture (default, 32 threads, no overlap) vs overlap vs HBM freeze,
# two rounds interleaved in one box call.
set -o pipefail
O=${OUT:-gpurun_out/r6/uvmcap6}
mkdir -p $O
export PYTHONUNBUFFERED=1 HSBENCH_DIR=$PWD/bench_tmp
mkdir -p $HSBENCH_DIR
for i in 1 2; do
for mode in "uvm_capture_overlap=False" "uvm_capture_overlap=True" "uvm_async_capture=False"; do
  for gb in 12.5 8; do
    tag=$(echo $mode | tr ' =' '_-')_${gb}gb_$i
    sp=""; [ $gb = 12.5 ] && sp="--single-path"
    timeout -k 10 300 python scripts/probes/with_tuning.py $mode -- benchmarks/dlrm_uvm/main.py --total-gb $gb --uvm --sync-repeats 3 $sp > $O/$tag.json 2> $O/$tag.err || { tail -20 $O/$tag.err; exit 1; }
    echo "$gb GB $mode: $(tail -1 $O/$tag.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ("sync_GBps","freeze_gpu_ms","async_total_s","async_GBps","restore_bitwise_ok")}, d["uvm_capture_stats"].get("copy_s"))')"
  done
done
done
