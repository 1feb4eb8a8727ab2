#!/bin/bash
# full GPU suite, smoke, headline bench, train-overlap benchmark (hsz1 + raw)
set -o pipefail
mkdir -p gpurun_out/overlap
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD:$PYTHONPATH HSBENCH_DIR=$PWD/bench_tmp
mkdir -p $HSBENCH_DIR
TESTS=1 STEPS=5 bash scripts/gpu_check.sh || exit 1
for c in hsz1 none; do
timeout -k 10 600 python benchmarks/train_overlap/main.py --seq 2048 --compression $c \
    > gpurun_out/overlap/fs_8b_$c.json 2> gpurun_out/overlap/fs_8b_$c.err \
    || { echo OVERLAP_FAIL; grep -v "^frame" gpurun_out/overlap/fs_8b_$c.err | tail -30; exit 1; }
tail -1 gpurun_out/overlap/fs_8b_$c.json
done
