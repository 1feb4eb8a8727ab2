#!/bin/bash
# Drain helper process: its GPU tests first, then the full GPU suite, smoke and
# the headline bench, then the seq-512 training overlap with the drain in
# process vs in the helper (interleaved, twice each).
set -o pipefail
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD HIPSNAPSHOT_BENCH_DIR=$PWD/bench_tmp
O=$PWD/gpurun_out/r3helper
mkdir -p $O bench_tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -v -m gpu -k "drain_process or native_drain" \
    --timeout 120 --timeout-method thread > $O/pytest_helper.log 2>&1 \
    || { echo PYTEST_HELPER_FAIL; tail -40 $O/pytest_helper.log; exit 1; }
tail -2 $O/pytest_helper.log
TESTS=${TESTS:-1} STEPS=10 bash scripts/gpu_check.sh || exit 1
for i in 1 2; do
for v in inproc helper; do
  if [ $v = helper ]; then export HIPSNAPSHOT_DRAIN_PROCESS=1; else export HIPSNAPSHOT_DRAIN_PROCESS=0; fi
  timeout -k 10 400 python benchmarks/train_overlap/main.py --seq 512 --checkpoints 5 \
      --gap-steps 15 --window-steps 30 --compression hsz1 > $O/ov512_${v}_$i.json 2> $O/ov512_${v}_$i.err \
      || { echo OVERLAP_FAIL $v $i; tail -20 $O/ov512_${v}_$i.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/ov512_${v}_$i.json').read().strip().splitlines()[-1]);print('$v $i', {k:d.get(k) for k in ['baseline_step_ms','sync_take_s','async_unblock_ms','async_drain_s_each','slowdown_during_drain','train_time_lost_ms','train_time_lost_vs_sync_take','train_time_lost_local_ms','train_time_lost_local_vs_sync_take','slowdown_local_median_each']})"
done
done
rm -rf bench_tmp
