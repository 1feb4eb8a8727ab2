#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/overlap
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD:$PYTHONPATH HIPSNAPSHOT_BENCH_DIR=$PWD/bench_tmp
mkdir -p $HIPSNAPSHOT_BENCH_DIR
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
df -h . | tail -1
timeout -k 10 600 python benchmarks/train_overlap/main.py --seq 2048 --compression none \
    > gpurun_out/overlap/fs_8b_raw.json 2> gpurun_out/overlap/fs_8b_raw.err \
    || { echo OVERLAP_RAW_FAIL; grep -v "^frame" gpurun_out/overlap/fs_8b_raw.err | tail -30; exit 1; }
tail -1 gpurun_out/overlap/fs_8b_raw.json; grep phase gpurun_out/overlap/fs_8b_raw.err
timeout -k 10 600 python benchmarks/train_overlap/main.py --seq 2048 \
    > gpurun_out/overlap/fs_8b.json 2> gpurun_out/overlap/fs_8b.err \
    || { echo OVERLAP_FAIL; grep -v "^frame" gpurun_out/overlap/fs_8b.err | tail -30; exit 1; }
tail -1 gpurun_out/overlap/fs_8b.json
