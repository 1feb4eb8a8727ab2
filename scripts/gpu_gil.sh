#!/bin/bash
# Is the drain's slowdown of training GIL contention?  Training overlap with
# Python's default 5 ms thread switch interval vs 0.5 ms, interleaved.
set -o pipefail
mkdir -p gpurun_out/gil
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD:$PYTHONPATH HIPSNAPSHOT_BENCH_DIR=$PWD/bench_tmp
mkdir -p $HIPSNAPSHOT_BENCH_DIR
for i in 1 2 3; do
for si in 5 0.5; do
  timeout -k 10 280 python benchmarks/train_overlap/main.py --seq 2048 --compression hsz1 --switch-interval-ms $si \
      > gpurun_out/gil/si${si}_$i.json 2> gpurun_out/gil/si${si}_$i.err \
      || { echo FAIL $si $i; grep -v "^frame" gpurun_out/gil/si${si}_$i.err | tail -20; exit 1; }
  echo "si=$si run=$i $(tail -1 gpurun_out/gil/si${si}_$i.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["async_unblock_ms"], d["async_drain_s"], d["steps_during_drain"], d["baseline_step_ms"], d["step_ms_during_drain_mean"], d["slowdown_during_drain"])')"
done
done
