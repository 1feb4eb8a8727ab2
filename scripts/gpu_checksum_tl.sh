#!/bin/bash
# phase timelines of the headline bench (hsz1 takes, restore, then raw takes)
# with checksums on / off
set -o pipefail
out=gpurun_out/cksum_tl
rm -rf $out; mkdir -p $out
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD:$PYTHONPATH HIPSNAPSHOT_BENCH_DIR=$PWD/bench_tmp
mkdir -p $HIPSNAPSHOT_BENCH_DIR
for ck in 1 0; do
  HIPSNAPSHOT_CHECKSUM=$ck HIPSNAPSHOT_TIMELINE=$PWD/$out/ck$ck timeout -k 10 300 python bench.py --steps 2 --warmup 1 \
      --async-iters 1 --restore-iters 1 --raw-steps 3 > $out/bench_ck$ck.json 2> $out/bench_ck$ck.err \
      || { echo FAIL $ck; tail -20 $out/bench_ck$ck.err; exit 1; }
  tail -1 $out/bench_ck$ck.json | cut -c1-200
  grep raw $out/bench_ck$ck.err
done
ls $out
