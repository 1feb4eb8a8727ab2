#!/bin/bash
# async_take time-to-unblock on the current tree: timeline run + split-encoder A/B
set -o pipefail
mkdir -p gpurun_out/unblock
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD:$PYTHONPATH HIPSNAPSHOT_BENCH_DIR=$PWD/bench_tmp
mkdir -p $HIPSNAPSHOT_BENCH_DIR
ARGS="--steps 2 --warmup 1 --async-iters 6 --no-restore-check --raw-steps 0"
HIPSNAPSHOT_TIMELINE=$PWD/gpurun_out/unblock/t timeout -k 10 300 python bench.py $ARGS \
    > gpurun_out/unblock/tl.json 2> gpurun_out/unblock/tl.err \
    || { echo TL_FAIL; tail -30 gpurun_out/unblock/tl.err; exit 1; }
grep async gpurun_out/unblock/tl.err
for v in 0 1; do
HIPSNAPSHOT_SPLIT_ENCODE=$v timeout -k 10 300 python bench.py $ARGS \
    > gpurun_out/unblock/split$v.json 2> gpurun_out/unblock/split$v.err \
    || { echo AB_FAIL; tail -30 gpurun_out/unblock/split$v.err; exit 1; }
echo "split=$v"; grep async gpurun_out/unblock/split$v.err
done
ls gpurun_out/unblock | head -40
