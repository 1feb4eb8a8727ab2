#!/bin/bash
# Session 2, call G: helper-process drain writer count A/B at seq 512
# (8 / 4 / 2 writers), seq 2048 with the helper, and a timeline of the
# 100 GB UVM DLRM save (where do 5 s go).
set -o pipefail
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD HIPSNAPSHOT_BENCH_DIR=$PWD/bench_tmp
O=$PWD/gpurun_out/s2g
mkdir -p $O bench_tmp
show() {
  python -c "import json;d=json.loads(open('$1').read().strip().splitlines()[-1]);print('$2', {k:d.get(k) for k in ['baseline_step_ms','sync_take_s','async_unblock_ms','async_drain_s_each','steps_during_drain','slowdown_during_drain','train_time_lost_ms','train_time_lost_vs_sync_take','train_time_lost_local_ms','train_time_lost_local_vs_sync_take','slowdown_local_median_each']})"
}
for w in 4 2 8; do
  HIPSNAPSHOT_DRAIN_WRITERS=$w timeout -k 10 400 python benchmarks/train_overlap/main.py --seq 512 --checkpoints 5 \
      --gap-steps 15 --window-steps 30 --compression hsz1 > $O/ov512_helper_w$w.json 2> $O/ov512_helper_w$w.err \
      || { echo OVERLAP_FAIL $w; tail -20 $O/ov512_helper_w$w.err; exit 1; }
  show $O/ov512_helper_w$w.json "writers $w"
done
timeout -k 10 500 python benchmarks/train_overlap/main.py --seq 2048 --checkpoints 4 \
    --gap-steps 15 --window-steps 30 --compression hsz1 > $O/ov2048_helper.json 2> $O/ov2048_helper.err \
    || { echo OVERLAP2048_FAIL; tail -20 $O/ov2048_helper.err; exit 1; }
show $O/ov2048_helper.json "seq2048 helper"
mkdir -p $O/tl
HIPSNAPSHOT_TIMELINE=$O/tl/dlrm100 timeout -k 10 900 python benchmarks/dlrm_uvm/main.py --total-gb 100 --uvm --single-path \
    --work-dir /dev/shm > $O/dlrm_uvm_100gb.json 2> $O/dlrm_uvm_100gb.err \
    || { echo DLRM100_FAIL; tail -20 $O/dlrm_uvm_100gb.err; rm -rf /dev/shm/hs_dlrm; exit 1; }
tail -1 $O/dlrm_uvm_100gb.json
ls $O/tl | head
rm -rf /dev/shm/hs_dlrm bench_tmp
