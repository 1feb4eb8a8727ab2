#!/bin/bash
# GPU session: smoke, headline bench, microbench, rocprofv3 kernel stats.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
export PYTHONPATH=$PWD:$PYTHONPATH
export HIPSNAPSHOT_BENCH_DIR=$PWD/bench_tmp
mkdir -p $HIPSNAPSHOT_BENCH_DIR
STEPS=${STEPS:-3}
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -50 gpurun_out/smoke.log; exit 1; }
timeout -k 10 600 python bench.py --steps $STEPS --warmup 1 > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH_FAIL; tail -40 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json; tail -12 gpurun_out/bench.err
if [ "${MICRO:-1}" = "1" ]; then
timeout -k 10 300 python benchmarks/microbench.py --dir $PWD/hs_micro_tmp > gpurun_out/micro.jsonl 2> gpurun_out/micro.err || { echo MICRO_FAIL; tail -30 gpurun_out/micro.err; exit 1; }
cat gpurun_out/micro.jsonl
fi
if [ "${PROF:-1}" = "1" ]; then
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 1 --warmup 1 --async-iters 1 > gpurun_out/prof.log 2>&1 || { echo PROF_FAIL; tail -30 gpurun_out/prof.log; exit 1; }
find gpurun_out/prof -name "*stats*" | head
fi
