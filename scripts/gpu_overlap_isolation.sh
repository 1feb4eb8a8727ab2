#!/bin/bash
# Cross-process isolation of the training slowdown during a snapshot drain:
# one trainer process, then one load process at a time (scripts/overlap_isolation.py).
set -o pipefail
out=gpurun_out/iso
rm -rf $out; mkdir -p $out
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD:$PYTHONPATH HIPSNAPSHOT_BENCH_DIR=$PWD/bench_tmp
mkdir -p $HIPSNAPSHOT_BENCH_DIR
timeout -k 10 300 python scripts/overlap_isolation.py --role train --out $out --seconds ${TRAIN_S:-150} > $out/train.out 2> $out/train.err &
TP=$!
for w in ${LOADS:-none take_hsz1 take_raw d2h write encode encode_capped}; do
  timeout -k 10 120 python scripts/overlap_isolation.py --role drain --what $w --out $out --lead 2 --seconds 6 > $out/d_$w.out 2> $out/d_$w.err || { echo "FAIL $w"; tail -5 $out/d_$w.err; kill $TP; exit 1; }
  echo "done $w"
done
wait $TP || { echo "trainer failed"; tail -5 $out/train.err; exit 1; }
python scripts/overlap_isolation.py --role summarize --out $out
