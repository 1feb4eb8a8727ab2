#!/bin/bash
# Full GPU suite + bench with the split-stream bf16 encoder, then the
# training-overlap benchmark (hsz1) alternating split encoder on / off.
set -o pipefail
out=gpurun_out/split_overlap
mkdir -p $out
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD:$PYTHONPATH HIPSNAPSHOT_BENCH_DIR=$PWD/bench_tmp
mkdir -p $HIPSNAPSHOT_BENCH_DIR
TESTS=1 STEPS=10 bash scripts/gpu_check.sh || exit 1
for r in 1 2; do
  for sp in 1 0; do
    HIPSNAPSHOT_SPLIT_ENCODE=$sp timeout -k 10 600 python benchmarks/train_overlap/main.py --seq 2048 \
        --compression hsz1 > $out/overlap_split${sp}_r$r.json 2> $out/overlap_split${sp}_r$r.err \
        || { echo OVERLAP_FAIL; grep -v "^frame" $out/overlap_split${sp}_r$r.err | tail -30; exit 1; }
    echo "split=$sp run=$r"; tail -1 $out/overlap_split${sp}_r$r.json
  done
done
