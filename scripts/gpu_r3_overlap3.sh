#!/bin/bash
# Drain-thread priority A/B: nice 10 (default) vs 0, 6 checkpoints each,
# with cgroup CPU accounting and train_step spans in the timeline.
set -o pipefail
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD HIPSNAPSHOT_BENCH_DIR=$PWD/bench_tmp
O=$PWD/gpurun_out/r3g
mkdir -p $O/tl bench_tmp
(cat /sys/fs/cgroup/cpu.max; grep -E "Cpus_allowed_list" /proc/self/status; nproc) > $O/box.txt 2>&1 || true
timeout -k 10 200 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 150 --timeout-method thread \
    -k "native_drain or kept_hbm_arena" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for mode in nice10 nice0; do
  echo "== $mode"
  case $mode in
    nice10) envs="HIPSNAPSHOT_TIMELINE=$O/tl/ov";;
    nice0) envs="HIPSNAPSHOT_DRAIN_NICE=0";;
  esac
  env $envs timeout -k 10 500 python benchmarks/train_overlap/main.py --seq 512 --checkpoints 6 \
      --gap-steps 15 --window-steps 30 --compression hsz1 > $O/overlap_$mode.json 2> $O/overlap_$mode.err \
      || { echo OVERLAP_FAIL $mode; tail -20 $O/overlap_$mode.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/overlap_$mode.json').read().strip().splitlines()[-1]);print({k:d[k] for k in ['baseline_step_ms','baseline_step_ms_pre','baseline_step_ms_post','sync_take_s','async_unblock_ms_each','async_unblock_gc_ms_each','gc_ms_in_window','cgroup_cpu_in_window','async_drain_s_each','steps_during_drain','slowdown_during_drain','step_ms_during_drain_median','train_time_lost_ms','train_time_lost_vs_sync_take','step_ms_between_checkpoints_median']}); print(d['step_ms_during_drain_each'])"
done
rm -rf bench_tmp
