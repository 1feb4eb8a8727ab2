#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD:$PYTHONPATH HIPSNAPSHOT_BENCH_DIR=$PWD/bench_tmp
mkdir -p $HIPSNAPSHOT_BENCH_DIR
timeout -k 10 600 python bench.py --steps 3 --warmup 1 > gpurun_out/bench_a.json 2> gpurun_out/bench_a.err || { echo BENCH_A_FAIL; tail -40 gpurun_out/bench_a.err; exit 1; }
cat gpurun_out/bench_a.json; grep -E "step|async|restore|warmup" gpurun_out/bench_a.err
HIPSNAPSHOT_GPU_SLAB_GATHER=0 timeout -k 10 600 python bench.py --steps 3 --warmup 1 --async-iters 0 --no-restore-check > gpurun_out/bench_b.json 2> gpurun_out/bench_b.err || { echo BENCH_B_FAIL; tail -40 gpurun_out/bench_b.err; exit 1; }
cat gpurun_out/bench_b.json; grep -E "step|warmup" gpurun_out/bench_b.err
timeout -k 10 300 python benchmarks/microbench.py --skip-fs > gpurun_out/micro.jsonl 2> gpurun_out/micro.err || { echo MICRO_FAIL; tail -30 gpurun_out/micro.err; exit 1; }
cat gpurun_out/micro.jsonl
