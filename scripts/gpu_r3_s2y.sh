#!/bin/bash
# Session 2, call Y: timelines of bench.py's warm async_takes (what is left in
# the 5.5 ms unblock).
set -o pipefail
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD HIPSNAPSHOT_BENCH_DIR=$PWD/bench_tmp
O=$PWD/gpurun_out/s2y
mkdir -p $O/tl bench_tmp
HIPSNAPSHOT_TIMELINE=$O/tl/b timeout -k 10 300 python bench.py --steps 2 --warmup 1 --raw-steps 0 \
    --fresh-steps 0 --ddp-steps 0 --restore-iters 1 --async-iters 4 > $O/bench.json 2> $O/bench.err \
    || { echo BENCH_FAIL; tail -30 $O/bench.err; exit 1; }
grep async $O/bench.err
ls $O/tl | head -20
rm -rf bench_tmp
