#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r5/l
export PYTHONUNBUFFERED=1 HSBENCH_DIR=$PWD/bench_tmp
mkdir -p $HSBENCH_DIR
for i in 1 2 3; do
  PROBE_TL=gpurun_out/r5/l/tl$i timeout -k 10 300 python scripts/probes/cold_async_profile.py > gpurun_out/r5/l/plain$i.log 2>&1 || exit 1
done
grep -h cold_unblock gpurun_out/r5/l/plain*.log
for i in 1 2 3; do python scripts/probes/timeline_sum.py gpurun_out/r5/l/tl$i.rank0.async_take0; done
