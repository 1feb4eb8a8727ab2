#!/bin/bash
# headline bench (N = 1) + training-overlap benchmark on the current tree
set -o pipefail
out=gpurun_out/final1
mkdir -p $out bench_tmp
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD:$PYTHONPATH HIPSNAPSHOT_BENCH_DIR=$PWD/bench_tmp
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > $out/bench.json 2> $out/bench.err \
    || { echo FAIL bench; tail -20 $out/bench.err; exit 1; }
tail -1 $out/bench.json | cut -c1-250
grep -E "^async|^restore|^raw" $out/bench.err
timeout -k 10 300 python benchmarks/train_overlap/main.py --seq 2048 --compression hsz1 \
    > $out/overlap.json 2> $out/overlap.err || { echo FAIL overlap; tail -20 $out/overlap.err; exit 1; }
tail -1 $out/overlap.json
