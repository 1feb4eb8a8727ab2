#!/bin/bash
# Drain under GPU load (hash on/off), then the overlap at seq 2048 and 512
# with the GC-after-plan change.
set -o pipefail
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD HIPSNAPSHOT_BENCH_DIR=$PWD/bench_tmp
O=$PWD/gpurun_out/r3j
mkdir -p $O bench_tmp
timeout -k 10 300 python scripts/drain_contention_probe.py --gb 8 > $O/drain_probe.jsonl 2> $O/drain_probe.err \
    || { echo PROBE_FAIL; tail -20 $O/drain_probe.err; exit 1; }
cat $O/drain_probe.jsonl
for seq in 2048 512; do
  echo "== seq $seq"
  timeout -k 10 500 python benchmarks/train_overlap/main.py --seq $seq --checkpoints 5 \
      --gap-steps 15 --window-steps 30 --compression hsz1 > $O/overlap_seq$seq.json 2> $O/overlap_seq$seq.err \
      || { echo OVERLAP_FAIL $seq; tail -20 $O/overlap_seq$seq.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/overlap_seq$seq.json').read().strip().splitlines()[-1]);print({k:d[k] for k in ['baseline_step_ms','sync_take_s','cold_async_unblock_ms','cold_async_total_s','async_unblock_ms_each','async_unblock_gc_ms_each','async_drain_s_each','slowdown_during_drain','step_ms_during_drain_median','step_ms_between_checkpoints_median','train_time_lost_ms','train_time_lost_vs_sync_take','train_time_lost_local_ms','train_time_lost_local_vs_sync_take','train_time_lost_local_ms_each','restore_bitwise_ok']})"
done
rm -rf bench_tmp
