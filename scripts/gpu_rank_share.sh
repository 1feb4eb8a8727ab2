#!/bin/bash
# per-rank share of the Llama-3-8B save at W = 1, 2, 4, 8 on one GPU (what
# the fixed per-take costs do to scaling), plus one timeline at W = 8
set -o pipefail
out=gpurun_out/rank_share
mkdir -p $out
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD:$PYTHONPATH HSBENCH_DIR=$PWD/bench_tmp
mkdir -p $HSBENCH_DIR
for w in ${WS:-8 4 2 1}; do
  for c in ${COMP:-hsz1 none}; do
    timeout -k 10 240 python benchmarks/rank_share/main.py --world $w --compression $c \
        > $out/w${w}_$c.json 2> $out/w${w}_$c.err || { echo FAIL $w $c; tail -20 $out/w${w}_$c.err; exit 1; }
    cat $out/w${w}_$c.json
  done
done
HIPSNAPSHOT_TIMELINE=$PWD/$out/tl8 timeout -k 10 240 python benchmarks/rank_share/main.py --world 8 \
    --steps 3 --warmup 2 --async-iters 2 --restore-iters 1 > $out/tl8.json 2> $out/tl8.err \
    || { echo FAIL tl; tail -20 $out/tl8.err; exit 1; }
ls $out | head -40
timeout -k 10 300 python bench.py --steps 5 --warmup 2 > $out/bench.json 2> $out/bench.err || { echo FAIL bench; tail -20 $out/bench.err; exit 1; }; tail -1 $out/bench.json
