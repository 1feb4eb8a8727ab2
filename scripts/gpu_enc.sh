#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -v -m gpu -k "hsz or compressed" --timeout 120 \
    --timeout-method thread > gpurun_out/pytest_hsz.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_hsz.log; exit 1; }
tail -1 gpurun_out/pytest_hsz.log
timeout -k 10 300 python benchmarks/microbench.py --skip-fs > gpurun_out/micro.jsonl 2> gpurun_out/micro.err \
    || { echo MICRO_FAIL; tail -30 gpurun_out/micro.err; exit 1; }
grep hsz gpurun_out/micro.jsonl
