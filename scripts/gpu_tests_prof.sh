#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 900 python -m pytest tests -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_gpu.log
grep -E "^FAILED" gpurun_out/pytest_gpu.log | head -20
timeout -k 10 120 python scripts/probe_f64_f16.py
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_micro -o micro -- python3 benchmarks/microbench.py --skip-fs > gpurun_out/micro.jsonl 2> gpurun_out/micro.err || { echo MICRO_FAIL; tail -20 gpurun_out/micro.err; exit 1; }
cat gpurun_out/micro.jsonl
