#!/bin/bash
# HSZ1 mode-2 kernels first (bit-exact vs the NumPy reference), then the whole
# GPU suite, smoke and the headline bench.  Stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -v -m gpu -k "hsz" --timeout 120 \
    --timeout-method thread > gpurun_out/pytest_hsz.log 2>&1 \
    || { echo HSZ_FAIL; tail -40 gpurun_out/pytest_hsz.log; exit 1; }
tail -2 gpurun_out/pytest_hsz.log
exec_rest() { bash scripts/gpu_check.sh; }
exec_rest
