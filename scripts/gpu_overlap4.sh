#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/overlap
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD:$PYTHONPATH HIPSNAPSHOT_BENCH_DIR=$PWD/bench_tmp
mkdir -p $HIPSNAPSHOT_BENCH_DIR
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -v -m gpu -k "async" --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_async.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_async.log; exit 1; }
tail -1 gpurun_out/pytest_async.log
timeout -k 10 600 python benchmarks/train_overlap/main.py --seq 2048 --compression none \
    > gpurun_out/overlap/fs_8b_raw.json 2> gpurun_out/overlap/fs_8b_raw.err \
    || { echo OVERLAP_RAW_FAIL; grep -v "^frame" gpurun_out/overlap/fs_8b_raw.err | tail -30; exit 1; }
tail -1 gpurun_out/overlap/fs_8b_raw.json
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_overlap -o ov \
    -- python3 benchmarks/train_overlap/main.py --seq 2048 --baseline-steps 3 \
    > gpurun_out/overlap/fs_8b_prof.json 2> gpurun_out/overlap/fs_8b_prof.err \
    || { echo PROF_FAIL; grep -v "^frame" gpurun_out/overlap/fs_8b_prof.err | tail -30; exit 1; }
tail -1 gpurun_out/overlap/fs_8b_prof.json
