#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/overlap
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD:$PYTHONPATH HIPSNAPSHOT_BENCH_DIR=$PWD/bench_tmp
mkdir -p $HIPSNAPSHOT_BENCH_DIR
timeout -k 10 600 python benchmarks/train_overlap/main.py --seq 2048 --compression none \
    > gpurun_out/overlap/fs_8b_raw.json 2> gpurun_out/overlap/fs_8b_raw.err \
    || { echo OVERLAP_FAIL; tail -30 gpurun_out/overlap/fs_8b_raw.err; exit 1; }
tail -1 gpurun_out/overlap/fs_8b_raw.json
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d gpurun_out/prof_overlap -o ov \
    -- python3 benchmarks/train_overlap/main.py --seq 2048 --baseline-steps 3 \
    > gpurun_out/overlap/fs_8b_prof.json 2> gpurun_out/overlap/fs_8b_prof.err \
    || { echo PROF_FAIL; tail -30 gpurun_out/overlap/fs_8b_prof.err; exit 1; }
tail -1 gpurun_out/overlap/fs_8b_prof.json
