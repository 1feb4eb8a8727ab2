#!/bin/bash
# In-process interleaved A/B of the split-stream bf16 encoder on the take:
# one rank's share at W = 1 (the whole 8B model) and W = 8.
set -o pipefail
out=gpurun_out/split_take_ab
mkdir -p $out
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD:$PYTHONPATH HIPSNAPSHOT_BENCH_DIR=$PWD/bench_tmp
mkdir -p $HIPSNAPSHOT_BENCH_DIR
for w in 1 8; do
  timeout -k 10 400 python benchmarks/rank_share/main.py --world $w --steps 12 --warmup 2 \
      --async-iters 2 --restore-iters 3 --ab HIPSNAPSHOT_SPLIT_ENCODE=1,0 \
      > $out/w$w.json 2> $out/w$w.err || { echo FAIL $w; tail -20 $out/w$w.err; exit 1; }
  cat $out/w$w.json
done
