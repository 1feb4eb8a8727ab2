#!/bin/bash
# Ring-allocator check: native restore tests, W = 8 share, bench (cold and
# warm restore), then the rocprofv3 stats pass.
set -o pipefail
out=gpurun_out/s3c
mkdir -p $out
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD:$PYTHONPATH HSBENCH_DIR=$PWD/bench_tmp
mkdir -p $HSBENCH_DIR
timeout -k 10 300 python -u -m pytest tests/test_native_restore.py -x -q --timeout 120 \
    --timeout-method thread > $out/pytest_native.log 2>&1 || { tail -40 $out/pytest_native.log; exit 1; }
tail -1 $out/pytest_native.log
timeout -k 10 240 python benchmarks/rank_share/main.py --world 8 > $out/rs8.json 2> $out/rs8.err \
    || { echo RS_FAIL; tail -30 $out/rs8.err; exit 1; }
tail -1 $out/rs8.json | cut -c1-900
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --restore-iters 4 --raw-steps 0 \
    --fresh-steps 0 --ddp-steps 0 --ddp-llama-steps 0 > $out/bench.json 2> $out/bench.err \
    || { echo BENCH_FAIL; tail -30 $out/bench.err; exit 1; }
grep "^restore" $out/bench.err
bash scripts/gpu_prof_r4.sh
