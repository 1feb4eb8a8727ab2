#!/bin/bash
# Phase timeline of the 1-GPU Llama-3-8B restore (bench.py, hsz1): where the
# restore's time goes between page-cache reads, H2D and decode.
set -o pipefail
out=gpurun_out/restore_tl
mkdir -p $out
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD:$PYTHONPATH HSBENCH_DIR=$PWD/bench_tmp
mkdir -p $HSBENCH_DIR
HIPSNAPSHOT_TIMELINE=$PWD/$out/t timeout -k 10 300 python bench.py --steps 2 --warmup 1 \
    --async-iters 1 --restore-iters ${RESTORE_ITERS:-3} --raw-steps 0 ${BENCH_ARGS:-} \
    > $out/bench.json 2> $out/bench.err || { echo FAIL; tail -20 $out/bench.err; exit 1; }
cat $out/bench.json
ls $out | head -20
for f in $out/t.rank0.restore*.json; do python scripts/timeline_summary.py $f > ${f%.json}.txt; done
tail -25 $out/t.rank0.restore0.txt
