#!/bin/bash
# GPU tests touching the copy-descriptor changes, then the train-overlap benchmark.
set -o pipefail
mkdir -p gpurun_out/overlap
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD:$PYTHONPATH HIPSNAPSHOT_BENCH_DIR=$PWD/bench_tmp
mkdir -p $HIPSNAPSHOT_BENCH_DIR
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 600 python benchmarks/train_overlap/main.py --seq 2048 \
    > gpurun_out/overlap/fs_8b.json 2> gpurun_out/overlap/fs_8b.err \
    || { echo OVERLAP_FAIL; tail -30 gpurun_out/overlap/fs_8b.err; exit 1; }
tail -1 gpurun_out/overlap/fs_8b.json
timeout -k 10 600 python benchmarks/train_overlap/main.py --seq 2048 --layers 4 --storage s3 \
    > gpurun_out/overlap/s3_8b_l4.json 2> gpurun_out/overlap/s3_8b_l4.err \
    || { echo OVERLAP_S3_FAIL; tail -30 gpurun_out/overlap/s3_8b_l4.err; exit 1; }
tail -1 gpurun_out/overlap/s3_8b_l4.json
