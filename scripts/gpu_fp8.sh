#!/bin/bash
# fp8 quantize / dequantize kernels: GPU tests (hadamard + fp8 + mx8), host-timed
# rates on 1 GiB of bf16 and rocprofv3 kernel stats.
set -o pipefail
mkdir -p gpurun_out/fp8
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q -k "hadamard or fp8 or mx8" --timeout 120 --timeout-method thread \
    > gpurun_out/fp8/pytest_hadamard.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/fp8/pytest_hadamard.log; exit 1; }
tail -2 gpurun_out/fp8/pytest_hadamard.log
timeout -k 10 300 python scripts/fp8_kernels_bench.py > gpurun_out/fp8/rates.jsonl 2>&1 \
    || { echo BENCH_FAIL; tail -20 gpurun_out/fp8/rates.jsonl; exit 1; }
cat gpurun_out/fp8/rates.jsonl
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fp8/prof -o fp8 \
    -- python3 scripts/fp8_kernels_bench.py hadamard32 none > gpurun_out/fp8/prof.log 2>&1 \
    || { echo PROF_FAIL; tail -20 gpurun_out/fp8/prof.log; exit 1; }
find gpurun_out/fp8/prof -name "*kernel_stats*" -exec cat {} \;
