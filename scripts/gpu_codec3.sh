#!/bin/bash
# codec kernels: bit-exact tests, microbench (+ rocprof kernel stats), then a
# timeline of take/restore of the headline bench.
set -o pipefail
mkdir -p gpurun_out/timeline
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD:$PYTHONPATH HIPSNAPSHOT_BENCH_DIR=$PWD/bench_tmp
mkdir -p $HIPSNAPSHOT_BENCH_DIR
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -v -m gpu -k "hsz or compressed" \
    --timeout 120 --timeout-method thread > gpurun_out/pytest_hsz.log 2>&1 \
    || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_hsz.log; exit 1; }
tail -1 gpurun_out/pytest_hsz.log
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_micro -o micro \
    -- python3 benchmarks/microbench.py --skip-fs > gpurun_out/micro.jsonl 2> gpurun_out/micro.err \
    || { echo MICRO_FAIL; tail -30 gpurun_out/micro.err; exit 1; }
grep hsz gpurun_out/micro.jsonl
HIPSNAPSHOT_TIMELINE=$PWD/gpurun_out/timeline/m2 timeout -k 10 600 python bench.py --steps 3 --warmup 1 --async-iters 1 \
    > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH_FAIL; tail -30 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json; grep -E "^step|restore" gpurun_out/bench.err
ls gpurun_out/timeline | head -20
