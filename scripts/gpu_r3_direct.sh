#!/bin/bash
# Native drain O_DIRECT: GPU tests, then the training overlap buffered vs
# O_DIRECT (seq 512), and buffered at seq 2048 (a less launch-bound step).
set -o pipefail
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD HIPSNAPSHOT_BENCH_DIR=$PWD/bench_tmp
O=$PWD/gpurun_out/r3i
mkdir -p $O bench_tmp
timeout -k 10 200 python -u -m pytest tests/test_gpu.py -m gpu -x -v --timeout 150 --timeout-method thread \
    -k "native_drain or kept_hbm_arena" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
grep -E "PASS|SKIP|FAIL" $O/tests.log | tail -6
for mode in direct buffered seq2048; do
  echo "== $mode"
  seq=512; envs=""
  case $mode in
    direct) envs="HIPSNAPSHOT_DRAIN_DIRECT_IO=1";;
    seq2048) seq=2048;;
  esac
  env $envs timeout -k 10 500 python benchmarks/train_overlap/main.py --seq $seq --checkpoints 5 \
      --gap-steps 15 --window-steps 30 --compression hsz1 > $O/overlap_$mode.json 2> $O/overlap_$mode.err \
      || { echo OVERLAP_FAIL $mode; tail -20 $O/overlap_$mode.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/overlap_$mode.json').read().strip().splitlines()[-1]);print({k:d[k] for k in ['baseline_step_ms','sync_take_s','async_unblock_ms_each','async_drain_s_each','slowdown_during_drain','step_ms_during_drain_median','step_ms_between_checkpoints_median','train_time_lost_ms','train_time_lost_vs_sync_take','train_time_lost_local_ms','train_time_lost_local_vs_sync_take','train_time_lost_local_ms_each','slowdown_local_median_each','restore_bitwise_ok']})"
done
rm -rf bench_tmp
