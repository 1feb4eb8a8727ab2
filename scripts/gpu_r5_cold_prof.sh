#!/bin/bash
# cold (fresh-process) restore: timeline + cProfile of its first and second restore
set -o pipefail
out=gpurun_out/cold_prof; mkdir -p $out
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD:$PYTHONPATH HSBENCH_DIR=$PWD/bench_tmp
mkdir -p $HSBENCH_DIR
timeout -k 10 400 python benchmarks/cold_restore/main.py > $out/cold.json 2> $out/cold.err \
    || { echo COLD_FAIL; tail -30 $out/cold.err; exit 1; }
cat $out/cold.json
HIPSNAPSHOT_TIMELINE=$PWD/$out/t timeout -k 10 400 python benchmarks/cold_restore/main.py \
    > $out/cold_tl.json 2> $out/cold_tl.err || { echo COLD_TL_FAIL; tail -30 $out/cold_tl.err; exit 1; }
cat $out/cold_tl.json
HSBENCH_PROFILE=$PWD/$out/prof timeout -k 10 400 python benchmarks/cold_restore/main.py \
    > $out/cold_prof.json 2> $out/cold_prof.err || { echo COLD_PROF_FAIL; tail -30 $out/cold_prof.err; exit 1; }
ls $out
