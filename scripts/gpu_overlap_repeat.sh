#!/bin/bash
# training-overlap benchmark repeated N times (run-to-run spread of the
# per-step slowdown while an async snapshot drains)
set -o pipefail
mkdir -p gpurun_out/overlap_rep
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD:$PYTHONPATH HSBENCH_DIR=$PWD/bench_tmp
mkdir -p $HSBENCH_DIR
for i in $(seq 1 ${N:-6}); do
  timeout -k 10 280 python benchmarks/train_overlap/main.py --seq 2048 --compression hsz1 \
      > gpurun_out/overlap_rep/run_$i.json 2> gpurun_out/overlap_rep/run_$i.err \
      || { echo FAIL $i; grep -v "^frame" gpurun_out/overlap_rep/run_$i.err | tail -20; exit 1; }
  echo "$i $(tail -1 gpurun_out/overlap_rep/run_$i.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["async_unblock_ms"], d["async_drain_s"], d["steps_during_drain"], d["baseline_step_ms"], d["step_ms_during_drain_mean"], d["slowdown_during_drain"], d["restore_bitwise_ok"])')"
done
