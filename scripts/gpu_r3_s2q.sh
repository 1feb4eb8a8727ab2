#!/bin/bash
# Session 2, call Q: in-process native drain with ONE release fence per drain
# (no per-chunk release event): drain GPU tests, then the seq-512 overlap x2.
set -o pipefail
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD HIPSNAPSHOT_BENCH_DIR=$PWD/bench_tmp
O=$PWD/gpurun_out/s2q
mkdir -p $O bench_tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -v -m gpu \
    -k "drain or kept_hbm or async or checksum" --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 \
    || { echo PYTEST_FAIL; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for i in 1 2; do
  timeout -k 10 400 python benchmarks/train_overlap/main.py --seq 512 --checkpoints 5 \
      --gap-steps 15 --window-steps 30 --compression hsz1 > $O/ov512_inproc_$i.json 2> $O/ov512_inproc_$i.err \
      || { echo OVERLAP_FAIL; tail -20 $O/ov512_inproc_$i.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/ov512_inproc_$i.json').read().strip().splitlines()[-1]);print({k:d.get(k) for k in ['baseline_step_ms','sync_take_s','async_unblock_ms','async_drain_s_each','slowdown_during_drain','train_time_lost_ms','train_time_lost_vs_sync_take','train_time_lost_local_vs_sync_take']}); print([ (s['sdma_submit'], s['wall']) for s in d.get('native_drain_stats_each') or []])"
done
rm -rf bench_tmp
