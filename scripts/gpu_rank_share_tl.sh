#!/bin/bash
# one timeline of the W-rank share take (default W = 8)
set -o pipefail
out=gpurun_out/rank_share_tl
rm -rf $out; mkdir -p $out
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD:$PYTHONPATH HSBENCH_DIR=$PWD/bench_tmp
mkdir -p $HSBENCH_DIR
for w in ${W:-8}; do
  HIPSNAPSHOT_TIMELINE=$PWD/$out/w$w timeout -k 10 240 python benchmarks/rank_share/main.py --world $w \
      --steps 4 --warmup 2 --async-iters 2 --restore-iters 1 > $out/w$w.json 2> $out/w$w.err \
      || { echo FAIL tl; tail -20 $out/w$w.err; exit 1; }
  tail -1 $out/w$w.json
done
