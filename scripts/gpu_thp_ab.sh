#!/bin/bash
# THP-backed registered pinned pool vs hipHostMalloc: GPU tests, then the
# headline bench and the 8-GPU share (take + restore), separate processes,
# interleaved
set -o pipefail
out=gpurun_out/thp_ab
mkdir -p $out bench_tmp
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD:$PYTHONPATH HIPSNAPSHOT_BENCH_DIR=$PWD/bench_tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread \
    > $out/tests.log 2>&1 || { echo FAIL tests; tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for i in 1 2; do for thp in 1 0; do
  HIPSNAPSHOT_PINNED_THP=$thp timeout -k 10 300 python bench.py --steps 6 --warmup 2 --raw-steps 2 \
      > $out/bench_thp${thp}_$i.json 2> $out/bench_thp${thp}_$i.err || { echo FAIL bench; tail $out/bench_thp${thp}_$i.err; exit 1; }
  echo "bench thp=$thp $i $(tail -1 $out/bench_thp${thp}_$i.json | python -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"], d["raw_GBps"], d["time_to_unblock_ms"], d["restore_GBps"], d["restore_GBps_each"])')"
  HIPSNAPSHOT_PINNED_THP=$thp timeout -k 10 200 python benchmarks/rank_share/main.py --world 8 --steps 10 --warmup 2 \
      --async-iters 2 --restore-iters 4 > $out/w8_thp${thp}_$i.json 2>/dev/null || { echo FAIL w8; exit 1; }
  echo "w8 thp=$thp $i $(tail -1 $out/w8_thp${thp}_$i.json | python -c 'import json,sys; d=json.load(sys.stdin); print(d["take_ms_median"], d["restore_ms_median"], d["unblock_ms_median"])')"
done; done
