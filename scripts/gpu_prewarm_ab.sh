#!/bin/bash
# first-restore A/B: HIPSNAPSHOT_RESTORE_PREWARM 0 / 1, alternating, bench.py
# (its restore_cold_GBps is the first restore of the process)
set -o pipefail
out=gpurun_out/prewarm_ab
mkdir -p $out
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD:$PYTHONPATH HSBENCH_DIR=$PWD/bench_tmp
mkdir -p $HSBENCH_DIR
timeout -k 10 400 python -u -m pytest tests/test_native_restore.py -x -q -m gpu --timeout 120 \
    --timeout-method thread > $out/tests.log 2>&1 || { echo TEST_FAIL; tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for i in 1 2; do
  for p in 0 1; do
    HIPSNAPSHOT_RESTORE_PREWARM=$p timeout -k 10 400 python bench.py --steps 2 --warmup 1 \
        > $out/bench_p${p}_$i.json 2> $out/bench_p${p}_$i.err || { echo BENCH_FAIL; tail -20 $out/bench_p${p}_$i.err; exit 1; }
    echo "prewarm=$p run $i: $(grep -o '"restore_cold_GBps": [0-9.]*' $out/bench_p${p}_$i.json) $(grep -o 'restore: [^{]*' $out/bench_p${p}_$i.err)"
  done
done
