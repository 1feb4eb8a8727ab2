#!/bin/bash
# Phase timelines of the W-rank share restore (default W = 8, hsz1): where the
# restore's time goes between planning, page-cache reads, H2D and decode.
set -o pipefail
out=gpurun_out/rs_restore_tl
rm -rf $out; mkdir -p $out
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD:$PYTHONPATH HSBENCH_DIR=$PWD/bench_tmp
mkdir -p $HSBENCH_DIR
W=${W:-8}
HIPSNAPSHOT_TIMELINE=$PWD/$out/t timeout -k 10 240 python benchmarks/rank_share/main.py --world $W \
    --steps 2 --warmup 1 --async-iters 1 --restore-iters ${RESTORE_ITERS:-4} \
    --compression ${COMP:-hsz1} > $out/w$W.json 2> $out/w$W.err \
    || { echo FAIL; tail -20 $out/w$W.err; exit 1; }
tail -1 $out/w$W.json
ls $out | head -40
for f in $out/t*restore*.json; do python scripts/timeline_summary.py $f > ${f%.json}.txt; done
for f in $out/t*restore*.txt; do echo "== $f"; cat $f; done | tail -120
