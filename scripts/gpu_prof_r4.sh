#!/bin/bash
# rocprofv3 kernel + memory-copy stats of the 1-GPU bench (take, async take,
# native restore), then a kernel-trace-only pass of the W = 8 share restore.
set -o pipefail
mkdir -p gpurun_out/prof_r4
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD:$PYTHONPATH HSBENCH_DIR=$PWD/bench_tmp
mkdir -p $HSBENCH_DIR
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv \
    -d gpurun_out/prof_r4/bench -o bench -- python3 bench.py --steps 2 --warmup 1 --async-iters 1 \
    --restore-iters 2 --raw-steps 0 --fresh-steps 0 --ddp-steps 0 --ddp-llama-steps 0 \
    > gpurun_out/prof_r4/bench.log 2>&1 || { echo PROF_FAIL; tail -20 gpurun_out/prof_r4/bench.log; exit 1; }
find gpurun_out/prof_r4 -name "*stats*.csv" | head
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv \
    -d gpurun_out/prof_r4/rs8 -o rs8 -- python3 benchmarks/rank_share/main.py --world 8 \
    --steps 2 --warmup 1 --async-iters 1 --restore-iters 3 \
    > gpurun_out/prof_r4/rs8.log 2>&1 || { echo PROF8_FAIL; tail -20 gpurun_out/prof_r4/rs8.log; exit 1; }
find gpurun_out/prof_r4 -name "*trace.csv" -size +20M -delete
ls -R gpurun_out/prof_r4 | head -30
