#!/bin/bash
# File-mapping path: its GPU tests, then a bench (timed takes rewrite one path).
set -o pipefail
mkdir -p gpurun_out/r5/j
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_filemap.py -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/r5/j/filemap_tests.log 2>&1 || { echo "filemap tests rc $?"; tail -60 gpurun_out/r5/j/filemap_tests.log; exit 1; }
tail -12 gpurun_out/r5/j/filemap_tests.log
timeout -k 10 400 python bench.py --steps 5 --warmup 2 > gpurun_out/r5/j/bench.log 2>&1 || { echo "bench rc $?"; tail -30 gpurun_out/r5/j/bench.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r5/j/bench.log | tail -5
