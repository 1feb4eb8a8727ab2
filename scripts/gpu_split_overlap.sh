#!/bin/bash
# Full GPU suite + bench with the split-stream bf16 encoder and split head
# reads; restore A/B (HIPSNAPSHOT_READ_HEAD_BYTES default vs 0); then the
# training-overlap benchmark (hsz1) alternating split encoder on / off.
set -o pipefail
out=gpurun_out/split_overlap
mkdir -p $out
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD:$PYTHONPATH HIPSNAPSHOT_BENCH_DIR=$PWD/bench_tmp
mkdir -p $HIPSNAPSHOT_BENCH_DIR
TESTS=1 STEPS=10 bash scripts/gpu_check.sh || exit 1
for r in 1 2; do
  for hb in 16777216 0; do
    HIPSNAPSHOT_READ_HEAD_BYTES=$hb timeout -k 10 300 python bench.py --steps 1 --warmup 1 \
        --async-iters 0 --raw-steps 0 --restore-iters 5 > $out/restore_head${hb}_r$r.json \
        2> $out/restore_head${hb}_r$r.err || { echo RESTORE_FAIL; tail -20 $out/restore_head${hb}_r$r.err; exit 1; }
    echo "head=$hb run=$r $(grep -o '"restore_GBps_each": [^]]*]' $out/restore_head${hb}_r$r.json)"
  done
done
for r in 1 2; do
  for sp in 1 0; do
    HIPSNAPSHOT_SPLIT_ENCODE=$sp timeout -k 10 600 python benchmarks/train_overlap/main.py --seq 2048 \
        --compression hsz1 > $out/overlap_split${sp}_r$r.json 2> $out/overlap_split${sp}_r$r.err \
        || { echo OVERLAP_FAIL; grep -v "^frame" $out/overlap_split${sp}_r$r.err | tail -30; exit 1; }
    echo "split=$sp run=$r"; tail -1 $out/overlap_split${sp}_r$r.json
  done
done
