#!/bin/bash
# Cold async unblock (plain x3, one with a timeline), GPU suite, bench.
set -o pipefail
mkdir -p gpurun_out/r5/m
export PYTHONUNBUFFERED=1 HSBENCH_DIR=$PWD/bench_tmp
mkdir -p $HSBENCH_DIR
for i in 1 2 3; do
  timeout -k 10 300 python scripts/probes/cold_async_profile.py > gpurun_out/r5/m/cold$i.log 2>&1 || exit 1
done
PROBE_TL=gpurun_out/r5/m/tl timeout -k 10 300 python scripts/probes/cold_async_profile.py > gpurun_out/r5/m/cold_tl.log 2>&1 || exit 1
grep -h cold_unblock gpurun_out/r5/m/cold*.log
python scripts/probes/timeline_sum.py gpurun_out/r5/m/tl.rank0.async_take0 | cut -c1-600
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5/m/gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r5/m/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/r5/m/bench.log 2>&1 || { tail -20 gpurun_out/r5/m/bench.log; exit 1; }
grep -E "^(warmup|step|async|raw|fresh|DDP)" gpurun_out/r5/m/bench.log | cut -c1-200; tail -1 gpurun_out/r5/m/bench.log | cut -c1-400
