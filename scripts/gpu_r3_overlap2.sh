#!/bin/bash
# Training overlap A/B (kept arena, baseline from every no-drain step, GC
# accounting); the default mode also records a timeline of every take.
set -o pipefail
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD HIPSNAPSHOT_BENCH_DIR=$PWD/bench_tmp
O=$PWD/gpurun_out/r3f
mkdir -p $O/tl bench_tmp
for mode in default slot64; do
  echo "== $mode"
  case $mode in
    default) envs="HIPSNAPSHOT_TIMELINE=$O/tl/ov";;
    slot64) envs="HIPSNAPSHOT_DRAIN_SLOT_BYTES=67108864";;
  esac
  env $envs timeout -k 10 400 python benchmarks/train_overlap/main.py --seq 512 --checkpoints 4 \
      --gap-steps 15 --window-steps 30 --compression hsz1 > $O/overlap_$mode.json 2> $O/overlap_$mode.err \
      || { echo OVERLAP_FAIL $mode; tail -20 $O/overlap_$mode.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/overlap_$mode.json').read().strip().splitlines()[-1]);print({k:d[k] for k in ['baseline_step_ms','baseline_step_ms_pre','baseline_step_ms_post','sync_take_s','async_unblock_ms_each','async_unblock_gc_ms_each','gc_ms_in_window','async_drain_s_each','steps_during_drain','slowdown_during_drain','train_time_lost_ms','train_time_lost_vs_sync_take','step_ms_between_checkpoints_median','cold_async_unblock_ms','cold_async_total_s']}); print(d['step_ms_during_drain_each'])"
done
rm -rf bench_tmp
