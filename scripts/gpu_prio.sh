#!/bin/bash
# copy/codec stream priority: GPU tests touching streams, then the training
# overlap benchmark with normal- and low-priority copy streams.
set -o pipefail
mkdir -p gpurun_out/prio
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD:$PYTHONPATH HIPSNAPSHOT_BENCH_DIR=$PWD/bench_tmp
mkdir -p $HIPSNAPSHOT_BENCH_DIR
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -v -m gpu -k "async or stream or ordered or compressed" \
    --timeout 120 --timeout-method thread > gpurun_out/prio/pytest.log 2>&1 \
    || { echo PYTEST_FAIL; grep -E "FAILED|Error" gpurun_out/prio/pytest.log | head; exit 1; }
tail -1 gpurun_out/prio/pytest.log
for p in normal low; do
HIPSNAPSHOT_COPY_STREAM_PRIORITY=$p timeout -k 10 600 python benchmarks/train_overlap/main.py --seq 2048 \
    --compression hsz1 > gpurun_out/prio/overlap_$p.json 2> gpurun_out/prio/overlap_$p.err \
    || { echo OVERLAP_FAIL $p; grep -v "^frame" gpurun_out/prio/overlap_$p.err | tail -20; exit 1; }
tail -1 gpurun_out/prio/overlap_$p.json
done
