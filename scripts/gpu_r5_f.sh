#!/bin/bash
set -o pipefail
export PYTHONUNBUFFERED=1 HSBENCH_DIR=$PWD/bench_tmp
mkdir -p $HSBENCH_DIR gpurun_out/r5/f
timeout -k 10 600 python scripts/probes/trim_probe_mp.py > gpurun_out/r5/f/trim_probe_mp.log 2>&1; echo "rc $?"
grep "mode=" gpurun_out/r5/f/trim_probe_mp.log
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu.py -k "verify" > gpurun_out/r5/f/verify_tests.log 2>&1; echo "rc $?"
tail -3 gpurun_out/r5/f/verify_tests.log
