#!/bin/bash
set -o pipefail
export PYTHONUNBUFFERED=1 HSBENCH_DIR=$PWD/bench_tmp
mkdir -p $HSBENCH_DIR gpurun_out/r5/d
timeout -k 10 500 python scripts/probes/keep_ab.py 0 > gpurun_out/r5/d/keep_ab.log 2>&1; echo "rc $?"
grep -E "keep=" gpurun_out/r5/d/keep_ab.log
