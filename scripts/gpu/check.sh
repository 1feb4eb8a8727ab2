#!/bin/bash
# One GPU call: the GPU test suite, smoke(), the headline bench, and (PROF=1)
# a rocprofv3 kernel + copy trace of the bench.  Every GPU step has its own
# time limit; the chain stops at the first failure.
#   OUT=gpurun_out/check TESTS=1 STEPS=5 BENCH_ARGS="..." PROF=0
set -o pipefail
O=${OUT:-gpurun_out/check}
mkdir -p $O
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD:$PYTHONPATH HSBENCH_DIR=$PWD/bench_tmp
mkdir -p $HSBENCH_DIR
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread \
      > $O/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest_gpu.log; exit 1; }
  tail -1 $O/pytest_gpu.log
fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
    || { echo SMOKE_FAIL; tail -30 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py --steps ${STEPS:-5} --warmup 2 ${BENCH_ARGS:-} > $O/bench.json 2> $O/bench.err \
    || { echo BENCH_FAIL; tail -30 $O/bench.err; exit 1; }
tail -1 $O/bench.json | cut -c1-1500
if [ "${PROF:-0}" = "1" ]; then
  cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
  timeout -k 10 600 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv \
      -d $O/prof_bench -o bench -- python3 bench.py --steps 2 --warmup 1 --async-iters 1 \
      > $O/prof_bench.log 2>&1 || { echo PROF_FAIL; tail -20 $O/prof_bench.log; exit 1; }
  find $O/prof_bench -name "*stats*"
fi
