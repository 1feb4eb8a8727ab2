#!/bin/bash
# Training-overlap slowdown measured with stream-local vs device-wide step
# syncs (a device-wide sync also waits for the drain's copy streams).
set -o pipefail
out=gpurun_out/overlap_sync
mkdir -p $out
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD:$PYTHONPATH HIPSNAPSHOT_BENCH_DIR=$PWD/bench_tmp
mkdir -p $HIPSNAPSHOT_BENCH_DIR
for i in 1 2; do
  for m in stream device; do
    timeout -k 10 280 python benchmarks/train_overlap/main.py --seq 2048 --compression hsz1 \
        --step-sync $m > $out/${m}_$i.json 2> $out/${m}_$i.err || { echo FAIL $m $i; tail -20 $out/${m}_$i.err; exit 1; }
    echo "$m $i $(tail -1 $out/${m}_$i.json)"
  done
done
