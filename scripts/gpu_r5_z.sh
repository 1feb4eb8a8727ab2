#!/bin/bash
# A/B of knobs.TUNING.stage_head_alone on one rank's W = 8 share (alternating, same box).
set -o pipefail
mkdir -p gpurun_out/r5/z
export PYTHONUNBUFFERED=1 HSBENCH_DIR=$PWD/bench_tmp
mkdir -p $HSBENCH_DIR
for i in 1 2 3; do
  for v in True False; do
    timeout -k 10 300 python scripts/probes/with_tuning.py stage_head_alone=$v -- benchmarks/rank_share/main.py --world 8 --steps 10 --warmup 2 --async-iters 0 --restore-iters 1 > gpurun_out/r5/z/$v$i.json 2> gpurun_out/r5/z/$v$i.err || { tail -5 gpurun_out/r5/z/$v$i.err; exit 1; }
    echo "$v$i $(tail -1 gpurun_out/r5/z/$v$i.json | grep -o '"take_ms_median": [0-9.]*, "take_ms_min": [0-9.]*')"
  done
done
