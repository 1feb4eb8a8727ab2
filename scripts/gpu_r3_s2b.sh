#!/bin/bash
# Session 2, call B: seq-512 training overlap with the drain in process vs in
# the helper process (interleaved, twice each); then BASELINE config 5's
# storage on one GPU: async_take to the (out-of-process) fake S3 while training.
set -o pipefail
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD HIPSNAPSHOT_BENCH_DIR=$PWD/bench_tmp
O=$PWD/gpurun_out/s2b
mkdir -p $O bench_tmp
show() {
  python -c "import json;d=json.loads(open('$1').read().strip().splitlines()[-1]);print('$2', {k:d.get(k) for k in ['baseline_step_ms','sync_take_s','async_unblock_ms','async_drain_s_each','steps_during_drain','slowdown_during_drain','train_time_lost_ms','train_time_lost_vs_sync_take','train_time_lost_local_ms','train_time_lost_local_vs_sync_take','slowdown_local_median_each']})"
}
for i in 1 2; do
for v in inproc helper; do
  if [ $v = helper ]; then export HIPSNAPSHOT_DRAIN_PROCESS=1; else export HIPSNAPSHOT_DRAIN_PROCESS=0; fi
  timeout -k 10 400 python benchmarks/train_overlap/main.py --seq 512 --checkpoints 5 \
      --gap-steps 15 --window-steps 30 --compression hsz1 > $O/ov512_${v}_$i.json 2> $O/ov512_${v}_$i.err \
      || { echo OVERLAP_FAIL $v $i; tail -20 $O/ov512_${v}_$i.err; exit 1; }
  show $O/ov512_${v}_$i.json "$v $i"
done
done
unset HIPSNAPSHOT_DRAIN_PROCESS
timeout -k 10 500 python benchmarks/train_overlap/main.py --seq 2048 --checkpoints 2 --storage s3 \
    --gap-steps 10 --window-steps 30 --compression hsz1 > $O/ov2048_s3.json 2> $O/ov2048_s3.err \
    || { echo OVERLAP_S3_FAIL; tail -20 $O/ov2048_s3.err; exit 1; }
show $O/ov2048_s3.json s3
rm -rf bench_tmp
