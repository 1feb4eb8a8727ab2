#!/bin/bash
# Kept HBM arena: GPU tests, then the training overlap A/B (default / slot64).
set -o pipefail
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD HIPSNAPSHOT_BENCH_DIR=$PWD/bench_tmp
O=$PWD/gpurun_out/r3e
mkdir -p $O bench_tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread \
    -k "kept_hbm_arena or native_drain or async" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for mode in default slot64; do
  echo "== $mode"
  case $mode in
    default) envs="";;
    slot64) envs="HIPSNAPSHOT_DRAIN_SLOT_BYTES=67108864";;
  esac
  env $envs timeout -k 10 400 python benchmarks/train_overlap/main.py --seq 512 --checkpoints 3 \
      --gap-steps 15 --window-steps 30 --compression hsz1 > $O/overlap_$mode.json 2> $O/overlap_$mode.err \
      || { echo OVERLAP_FAIL $mode; tail -20 $O/overlap_$mode.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/overlap_$mode.json').read().strip().splitlines()[-1]);print({k:d[k] for k in ['baseline_step_ms','sync_take_s','async_unblock_ms_each','async_drain_s_each','steps_during_drain','slowdown_during_drain','train_time_lost_ms','train_time_lost_vs_sync_take','step_ms_between_checkpoints_median','cold_async_unblock_ms','cold_async_total_s']}); print(d['step_ms_during_drain_each'])"
done
rm -rf bench_tmp
