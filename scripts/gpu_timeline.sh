#!/bin/bash
# full GPU suite + smoke + bench, then one bench run with the phase timeline
set -o pipefail
mkdir -p gpurun_out/timeline2
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD:$PYTHONPATH HSBENCH_DIR=$PWD/bench_tmp
mkdir -p $HSBENCH_DIR
TESTS=${TESTS:-1} STEPS=5 bash scripts/gpu_check.sh || exit 1
HIPSNAPSHOT_TIMELINE=$PWD/gpurun_out/timeline2/t timeout -k 10 600 python bench.py --steps 3 --warmup 1 \
    > gpurun_out/timeline2/bench.json 2> gpurun_out/timeline2/bench.err \
    || { echo BENCH_TL_FAIL; tail -30 gpurun_out/timeline2/bench.err; exit 1; }
cat gpurun_out/timeline2/bench.json
ls gpurun_out/timeline2 | head -20
