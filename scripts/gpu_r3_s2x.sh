#!/bin/bash
# Session 2, call X: the first async_take's GC pass moved to the commit thread:
# bench.py (cold unblock) and the training overlap (cold checkpoint cost).
set -o pipefail
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD HIPSNAPSHOT_BENCH_DIR=$PWD/bench_tmp
O=$PWD/gpurun_out/s2x
mkdir -p $O bench_tmp
timeout -k 10 300 python bench.py --steps 5 --warmup 2 > $O/bench.json 2> $O/bench.err \
    || { echo BENCH_FAIL; tail -30 $O/bench.err; exit 1; }
python -c "import json;d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]);print({k:d.get(k) for k in ['value','time_to_unblock_ms','cold_time_to_unblock_ms','async_total_ms','restore_bitwise_ok']})"
timeout -k 10 500 python benchmarks/train_overlap/main.py --seq 2048 --checkpoints 3 \
    --gap-steps 15 --window-steps 30 --compression hsz1 > $O/ov2048.json 2> $O/ov2048.err \
    || { echo OVERLAP_FAIL; tail -20 $O/ov2048.err; exit 1; }
python -c "import json;d=json.loads(open('$O/ov2048.json').read().strip().splitlines()[-1]);print({k:d.get(k) for k in ['baseline_step_ms','cold_async_unblock_ms','cold_async_total_s','async_unblock_ms_each','async_drain_s_each','train_time_lost_vs_sync_take','train_time_lost_local_vs_sync_take','async_unblock_gc_ms_each','gc_ms_in_window']})"
rm -rf bench_tmp
