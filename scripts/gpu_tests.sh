#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 900 python -m pytest tests -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -40 gpurun_out/pytest_gpu.log
exit $rc
