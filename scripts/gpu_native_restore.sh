#!/bin/bash
# Native restore check: its GPU tests, the whole GPU suite, the W = 8 share
# restore (hsz1 + raw) and the 1-GPU bench.  Every step has its own limit.
set -o pipefail
out=gpurun_out/native_restore
mkdir -p $out
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD:$PYTHONPATH HSBENCH_DIR=$PWD/bench_tmp
mkdir -p $HSBENCH_DIR
timeout -k 10 300 python -u -m pytest tests/test_native_restore.py -x -v --timeout 120 \
    --timeout-method thread > $out/pytest_native.log 2>&1 \
    || { echo NATIVE_TESTS_FAIL; tail -60 $out/pytest_native.log; exit 1; }
tail -3 $out/pytest_native.log
if [ "${FULL:-1}" = "1" ]; then
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread \
    > $out/pytest_gpu.log 2>&1 || { echo GPU_TESTS_FAIL; tail -60 $out/pytest_gpu.log; exit 1; }
tail -3 $out/pytest_gpu.log
fi
for c in hsz1 none; do
  timeout -k 10 240 python benchmarks/rank_share/main.py --world 8 --compression $c \
      > $out/rs8_$c.json 2> $out/rs8_$c.err || { echo RS_FAIL $c; tail -30 $out/rs8_$c.err; exit 1; }
  tail -1 $out/rs8_$c.json
done
timeout -k 10 400 python bench.py --steps 5 --warmup 2 > $out/bench.json 2> $out/bench.err \
    || { echo BENCH_FAIL; tail -30 $out/bench.err; exit 1; }
tail -1 $out/bench.json
