#!/bin/bash
# Training overlap: HSZ1 vs raw drains (SDMA D2H), interleaved on one box.
set -o pipefail
out=gpurun_out/overlap_raw
mkdir -p $out
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD:$PYTHONPATH HIPSNAPSHOT_BENCH_DIR=$PWD/bench_tmp
mkdir -p $HIPSNAPSHOT_BENCH_DIR
i=0
for c in none hsz1 none hsz1; do
  i=$((i + 1))
  f=$out/run${i}_$c
  timeout -k 10 280 python benchmarks/train_overlap/main.py --seq 2048 --compression $c \
      > $f.json 2> $f.err || { echo FAIL $c; tail -20 $f.err; exit 1; }
  echo "$c $(tail -1 $f.json)"
done
