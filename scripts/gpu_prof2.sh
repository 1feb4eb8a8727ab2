#!/bin/bash
# async-take tests, data-plane microbench (codec GB/s), rocprofv3 kernel stats of the bench.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD:$PYTHONPATH HIPSNAPSHOT_BENCH_DIR=$PWD/bench_tmp
mkdir -p $HIPSNAPSHOT_BENCH_DIR
{ df -h . /var/tmp /tmp /dev/shm; free -g; nproc; } > gpurun_out/box_info.txt 2>&1
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -v -m gpu -k "async or hsz or compressed" \
    --timeout 120 --timeout-method thread > gpurun_out/pytest_async.log 2>&1 \
    || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_async.log; exit 1; }
tail -2 gpurun_out/pytest_async.log
timeout -k 10 300 python benchmarks/microbench.py --dir $PWD/hs_micro_tmp > gpurun_out/micro.jsonl 2> gpurun_out/micro.err \
    || { echo MICRO_FAIL; tail -30 gpurun_out/micro.err; exit 1; }
grep hsz gpurun_out/micro.jsonl
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv \
    -d gpurun_out/prof_bench -o bench -- python3 bench.py --steps 2 --warmup 1 --async-iters 1 \
    > gpurun_out/prof_bench.log 2>&1 || { echo PROF_FAIL; tail -20 gpurun_out/prof_bench.log; exit 1; }
find gpurun_out/prof_bench -name "*stats*"
