#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r5/k
export PYTHONUNBUFFERED=1 HSBENCH_DIR=$PWD/bench_tmp
mkdir -p $HSBENCH_DIR
HIPSNAPSHOT_TIMELINE=gpurun_out/r5/k/bt timeout -k 10 400 python bench.py --steps 2 --warmup 2 --async-iters 0 --raw-steps 0 --fresh-steps 0 --ddp-steps 0 --ddp-llama-steps 0 --verify-iters 0 --elastic-iters 0 --restore-iters 1 > gpurun_out/r5/k/bench_tl.log 2>&1; rc=$?
grep -E "^(warmup|step)" gpurun_out/r5/k/bench_tl.log; echo "bench rc $rc"
python scripts/probes/timeline_sum.py gpurun_out/r5/k/bt.rank0.take > gpurun_out/r5/k/bench_tl_sum.txt 2>&1
cut -c1-900 gpurun_out/r5/k/bench_tl_sum.txt
rm -f gpurun_out/r5/k/bt.*restore*.json
