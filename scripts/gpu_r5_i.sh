#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r5/i
export PYTHONUNBUFFERED=1 HSBENCH_DIR=$PWD/bench_tmp
mkdir -p $HSBENCH_DIR
timeout -k 10 400 python scripts/probes/${PROBE:-filemap_persist_probe.py} > gpurun_out/r5/i/${PROBE:-filemap_persist_probe.py}.log 2>&1; echo "rc $?"
grep -v "amdgpu.ids" gpurun_out/r5/i/${PROBE:-filemap_persist_probe.py}.log | tail -20
