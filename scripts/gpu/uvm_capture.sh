#!/bin/bash
# Round 6: async takes of host-resident UVM tables captured
# by CPU threads while the trainer's stream waits on a gate.  GPU tests, the
# capture-rate probe, DLRM 8 GB and the config-4 share (12.5 GB).
set -o pipefail
O=${OUT:-gpurun_out/r6/uvmcap}
mkdir -p $O
export PYTHONUNBUFFERED=1 HSBENCH_DIR=$PWD/bench_tmp
mkdir -p $HSBENCH_DIR
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_uvm_capture.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
for mode in "uvm_async_capture=True uvm_capture_overlap=False" "uvm_async_capture=True uvm_capture_overlap=True" "uvm_async_capture=False"; do
  tag=$(echo $mode | tr ' =' '_-')_$i
  timeout -k 10 300 python scripts/probes/with_tuning.py $mode -- benchmarks/dlrm_uvm/main.py --total-gb ${GB:-8} --uvm --sync-repeats 3 ${DLRM_ARGS:-} > $O/$tag.json 2> $O/$tag.err || { tail -20 $O/$tag.err; exit 1; }
  echo "$mode: $(tail -1 $O/$tag.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ("sync_GBps","sync_GBps_each","async_unblock_ms","freeze_gpu_ms","async_total_s","async_GBps","uvm_capture_stats","restore_bitwise_ok")})')"
done
done
