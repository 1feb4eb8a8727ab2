#!/bin/bash
# Session 2, call R: seq-2048 training overlap with the one-fence drain
# (the drain took 11-14 s before), and bench.py (async_total with the fix).
set -o pipefail
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD HIPSNAPSHOT_BENCH_DIR=$PWD/bench_tmp
O=$PWD/gpurun_out/s2r
mkdir -p $O bench_tmp
timeout -k 10 500 python benchmarks/train_overlap/main.py --seq 2048 --checkpoints 5 \
    --gap-steps 15 --window-steps 30 --compression hsz1 > $O/ov2048.json 2> $O/ov2048.err \
    || { echo OVERLAP_FAIL; tail -20 $O/ov2048.err; exit 1; }
python -c "import json;d=json.loads(open('$O/ov2048.json').read().strip().splitlines()[-1]);print({k:d.get(k) for k in ['baseline_step_ms','sync_take_s','async_unblock_ms','async_drain_s_each','slowdown_during_drain','train_time_lost_ms','train_time_lost_vs_sync_take','train_time_lost_local_vs_sync_take']}); print([ (s['sdma_submit'], s['wall'], s['pwrite'], s['slot_wait'], s['sdma_wait']) for s in d.get('native_drain_stats_each') or []])"
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > $O/bench.json 2> $O/bench.err \
    || { echo BENCH_FAIL; tail -30 $O/bench.err; exit 1; }
tail -1 $O/bench.json; grep -E "async" $O/bench.err
rm -rf bench_tmp
