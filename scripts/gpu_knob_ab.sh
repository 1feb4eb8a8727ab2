#!/bin/bash
# in-process interleaved A/B of a knob on one rank's share: AB="NAME=v1,v2" WS="8 1"
set -o pipefail
out=gpurun_out/knob_ab; mkdir -p $out
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD:$PYTHONPATH HIPSNAPSHOT_BENCH_DIR=$PWD/bench_tmp
mkdir -p $HIPSNAPSHOT_BENCH_DIR
tag=$(echo "$AB" | tr '=,' '__')
for w in ${WS:-8 1}; do for c in ${COMP:-hsz1}; do
  timeout -k 10 300 python benchmarks/rank_share/main.py --world $w --compression $c --steps ${STEPS:-25} --warmup 2 \
      --async-iters 1 --restore-iters ${RITERS:-1} --ab "$AB" > $out/${tag}_w${w}_$c.json 2> $out/${tag}_w${w}_$c.err \
      || { echo FAIL; tail $out/${tag}_w${w}_$c.err; exit 1; }
  grep "rank_share_ab\|rank_share_restore_ab" $out/${tag}_w${w}_$c.json
done; done
