#!/bin/bash
# HIP API + kernel trace statistics of the W = 8 share's take and restore
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
out=gpurun_out/prof_rs; rm -rf $out; mkdir -p $out
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD:$PYTHONPATH HSBENCH_DIR=$PWD/bench_tmp
mkdir -p $HSBENCH_DIR
timeout -k 10 400 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace --stats --output-format csv -d $out -o run -- \
    python benchmarks/rank_share/main.py --world ${W:-8} --steps 3 --warmup 1 --async-iters 0 --restore-iters 3 \
    > $out/stdout.txt 2> $out/stderr.txt || { echo FAIL; tail -20 $out/stderr.txt; exit 1; }
tail -1 $out/stdout.txt
find $out -name "*stats.csv" | head
