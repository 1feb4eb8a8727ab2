#!/bin/bash
# Session 2, call K: bench.py with the drain helper on (dedicated arena
# allocation, interim mapping reply + 30 s mapping timeout), then the helper's
# GPU tests and the seq-512 overlap with the helper.
set -o pipefail
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD HIPSNAPSHOT_BENCH_DIR=$PWD/bench_tmp
O=$PWD/gpurun_out/s2k
mkdir -p $O bench_tmp
HIPSNAPSHOT_DRAIN_PROCESS=1 HIPSNAPSHOT_DRAIN_HELPER_DEBUG=1 \
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 > $O/bench.json 2> $O/bench.err \
  || { echo BENCH_FAIL; grep -v "^frame" $O/bench.err | tail -30; exit 1; }
grep -E "hsdrain|async|drain" $O/bench.err | tail -24
tail -1 $O/bench.json
HIPSNAPSHOT_DRAIN_PROCESS=1 timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -v -m gpu \
    -k "drain_process or native_drain or kept_hbm or async" --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 \
    || { echo PYTEST_FAIL; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
HIPSNAPSHOT_DRAIN_PROCESS=1 timeout -k 10 400 python benchmarks/train_overlap/main.py --seq 512 --checkpoints 5 \
    --gap-steps 15 --window-steps 30 --compression hsz1 > $O/ov512_helper.json 2> $O/ov512_helper.err \
    || { echo OVERLAP_FAIL; tail -20 $O/ov512_helper.err; exit 1; }
python -c "import json;d=json.loads(open('$O/ov512_helper.json').read().strip().splitlines()[-1]);print({k:d.get(k) for k in ['baseline_step_ms','sync_take_s','async_unblock_ms','cold_async_total_s','async_drain_s_each','slowdown_during_drain','train_time_lost_ms','train_time_lost_vs_sync_take','train_time_lost_local_vs_sync_take']})"
rm -rf bench_tmp
