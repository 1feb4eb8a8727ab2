#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 300 python benchmarks/microbench.py --skip-fs > gpurun_out/micro.jsonl 2> gpurun_out/micro.err \
    || { echo MICRO_FAIL; tail -30 gpurun_out/micro.err; exit 1; }
grep -E "copy_nd|freeze|hsz" gpurun_out/micro.jsonl
