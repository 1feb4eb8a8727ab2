#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/overlap
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD:$PYTHONPATH HIPSNAPSHOT_BENCH_DIR=$PWD/bench_tmp
mkdir -p $HIPSNAPSHOT_BENCH_DIR
for q in 4 8 16; do
GPU_MAX_HW_QUEUES=$q timeout -k 10 600 python benchmarks/train_overlap/main.py --seq 2048 \
    > gpurun_out/overlap/hwq$q.json 2> gpurun_out/overlap/hwq$q.err \
    || { echo OVERLAP_FAIL; grep -v "^frame" gpurun_out/overlap/hwq$q.err | tail -30; exit 1; }
echo "hwq=$q $(tail -1 gpurun_out/overlap/hwq$q.json | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['async_unblock_ms'],d['async_drain_s'],d['steps_during_drain'],d['baseline_step_ms'],d['step_ms_during_drain_mean'],d['slowdown_during_drain'])")"
done
