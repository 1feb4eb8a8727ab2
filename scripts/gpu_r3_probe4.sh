#!/bin/bash
# Drain under GPU load: hash stream at default vs high priority; then the
# seq-2048 overlap and the native drain GPU tests.
set -o pipefail
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD HIPSNAPSHOT_BENCH_DIR=$PWD/bench_tmp
O=$PWD/gpurun_out/r3k
mkdir -p $O bench_tmp
timeout -k 10 200 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 150 --timeout-method thread \
    -k "native_drain or kept_hbm_arena or checksum" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python scripts/drain_contention_probe.py --gb 8 > $O/drain_probe.jsonl 2> $O/drain_probe.err \
    || { echo PROBE_FAIL; tail -20 $O/drain_probe.err; exit 1; }
cat $O/drain_probe.jsonl
timeout -k 10 500 python benchmarks/train_overlap/main.py --seq 2048 --checkpoints 5 \
    --gap-steps 15 --window-steps 30 --compression hsz1 > $O/overlap_seq2048.json 2> $O/overlap_seq2048.err \
    || { echo OVERLAP_FAIL; tail -20 $O/overlap_seq2048.err; exit 1; }
python -c "import json;d=json.loads(open('$O/overlap_seq2048.json').read().strip().splitlines()[-1]);print({k:d[k] for k in ['baseline_step_ms','sync_take_s','cold_async_unblock_ms','async_unblock_ms_each','async_drain_s_each','slowdown_during_drain','train_time_lost_ms','train_time_lost_vs_sync_take','train_time_lost_local_ms','train_time_lost_local_vs_sync_take','restore_bitwise_ok']})"
rm -rf bench_tmp
