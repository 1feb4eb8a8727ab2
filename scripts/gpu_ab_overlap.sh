#!/bin/bash
# A/B of the training-overlap benchmark: current tree vs ab_old/ (an older
# commit's package + benchmark, built in-tree), interleaved, twice each.
set -o pipefail
mkdir -p gpurun_out/ab
export PYTHONUNBUFFERED=1 HIPSNAPSHOT_BENCH_DIR=$PWD/bench_tmp
mkdir -p $HIPSNAPSHOT_BENCH_DIR
for i in 1 2; do
for v in new old; do
  if [ $v = new ]; then S=benchmarks/train_overlap/main.py; else S=ab_old/benchmarks/train_overlap/main.py; fi
  timeout -k 10 280 python $S --seq 2048 --compression hsz1 > gpurun_out/ab/${v}_$i.json 2> gpurun_out/ab/${v}_$i.err \
      || { echo FAIL $v $i; grep -v "^frame" gpurun_out/ab/${v}_$i.err | tail -20; exit 1; }
  echo "$v $i $(tail -1 gpurun_out/ab/${v}_$i.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["async_unblock_ms"], d["async_drain_s"], d["steps_during_drain"], d["baseline_step_ms"], d["step_ms_during_drain_mean"], d["slowdown_during_drain"])')"
done
done
