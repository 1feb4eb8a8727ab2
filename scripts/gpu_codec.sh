#!/bin/bash
# Compression path on the GPU: tests, then the headline bench raw vs hsz1.
set -o pipefail
mkdir -p gpurun_out/timeline
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD:$PYTHONPATH HIPSNAPSHOT_BENCH_DIR=$PWD/bench_tmp
mkdir -p $HIPSNAPSHOT_BENCH_DIR
timeout -k 10 600 python -m pytest tests/test_gpu.py -q -x -k "hsz or compressed" > gpurun_out/codec_tests.log 2>&1 || { echo CODEC_TEST_FAIL; tail -40 gpurun_out/codec_tests.log; exit 1; }
tail -1 gpurun_out/codec_tests.log
for c in none hsz1; do
  HIPSNAPSHOT_TIMELINE=$PWD/gpurun_out/timeline/$c timeout -k 10 400 python bench.py --steps 5 --warmup 2 --async-iters 2 --compression $c > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err || { echo BENCH_FAIL $c; tail -30 gpurun_out/bench_$c.err; exit 1; }
  cat gpurun_out/bench_$c.json; grep -E "^step|^async|^restore" gpurun_out/bench_$c.err
  python scripts/timeline_summary.py gpurun_out/timeline/$c.rank0.take6.json gpurun_out/timeline/$c.rank0.restore0.json > gpurun_out/timeline_$c.txt 2>&1; cat gpurun_out/timeline_$c.txt
done
