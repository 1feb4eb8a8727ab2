#!/bin/bash
# Iteration loop: GPU tests, headline bench + timeline, FSDP bench + timeline.
set -o pipefail
mkdir -p gpurun_out/timeline
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD:$PYTHONPATH HIPSNAPSHOT_BENCH_DIR=$PWD/bench_tmp
mkdir -p $HIPSNAPSHOT_BENCH_DIR
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 900 python -m pytest tests -q -m gpu -x > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
  tail -1 gpurun_out/pytest_gpu.log
fi
HIPSNAPSHOT_TIMELINE=$PWD/gpurun_out/timeline/b timeout -k 10 400 python bench.py --steps 5 --warmup 2 --async-iters 2 > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH_FAIL; tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json; grep -E "^step|^async|^restore" gpurun_out/bench.err
python scripts/timeline_summary.py gpurun_out/timeline/b.rank0.take6.json gpurun_out/timeline/b.rank0.restore0.json > gpurun_out/timeline_summary.txt 2>&1; cat gpurun_out/timeline_summary.txt
HIPSNAPSHOT_TIMELINE=$PWD/gpurun_out/timeline/f timeout -k 10 400 python benchmarks/fsdp/main.py > gpurun_out/fsdp.json 2> gpurun_out/fsdp.err || { echo FSDP_FAIL; tail -20 gpurun_out/fsdp.err; exit 1; }
cat gpurun_out/fsdp.json
python scripts/timeline_summary.py gpurun_out/timeline/f.rank0.restore0.json > gpurun_out/timeline_fsdp.txt 2>&1; cat gpurun_out/timeline_fsdp.txt
