#!/bin/bash
# Host-contended rank-share rehearsal at W = 2 / 4 (W = 8 in profiles/r3/rank_share),
# then the training overlap with the local-baseline accounting.
set -o pipefail
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD HIPSNAPSHOT_BENCH_DIR=$PWD/bench_tmp
O=$PWD/gpurun_out/r3h
mkdir -p $O bench_tmp
for w in 2 4; do
  s=$((w - 1))
  timeout -k 10 400 python benchmarks/rank_share/main.py --world $w --steps 10 --warmup 3 --async-iters 3 \
      --restore-iters 2 --host-siblings $s --sibling-dma-pass 1 > $O/rank_share_w${w}_sib$s.json \
      2> $O/rank_share_w${w}_sib$s.err || { echo RANKSHARE_FAIL $w; tail -20 $O/rank_share_w${w}_sib$s.err; exit 1; }
  tail -1 $O/rank_share_w${w}_sib$s.json
done
timeout -k 10 500 python benchmarks/train_overlap/main.py --seq 512 --checkpoints 6 \
    --gap-steps 15 --window-steps 30 --compression hsz1 > $O/overlap.json 2> $O/overlap.err \
    || { echo OVERLAP_FAIL; tail -20 $O/overlap.err; exit 1; }
python -c "import json;d=json.loads(open('$O/overlap.json').read().strip().splitlines()[-1]);print({k:d[k] for k in ['baseline_step_ms','sync_take_s','async_unblock_ms_each','async_unblock_gc_ms_each','slowdown_during_drain','train_time_lost_ms','train_time_lost_vs_sync_take','train_time_lost_local_ms','train_time_lost_local_vs_sync_take','train_time_lost_local_ms_each','slowdown_local_median_each']})"
rm -rf bench_tmp
