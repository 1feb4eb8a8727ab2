#!/bin/bash
set -o pipefail
export PYTHONUNBUFFERED=1 HSBENCH_DIR=$PWD/bench_tmp
mkdir -p $HSBENCH_DIR gpurun_out/r5/e
timeout -k 10 300 python scripts/probes/trim_probe.py > gpurun_out/r5/e/trim_probe.log 2>&1; echo "rc $?"
grep -v "^RCCL\|^HIP\|^ROCm\|^Host\|^Librccl\|amdgpu.ids" gpurun_out/r5/e/trim_probe.log | tail -30
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu.py -k "verify" > gpurun_out/r5/e/verify_tests.log 2>&1; echo "rc $?"
tail -5 gpurun_out/r5/e/verify_tests.log
