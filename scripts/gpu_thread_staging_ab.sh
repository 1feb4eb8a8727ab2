#!/bin/bash
# thread-driven staging (default) vs one event-loop round trip per request,
# interleaved: one rank's share at W = 8 and W = 1, then the headline bench
set -o pipefail
out=gpurun_out/tstage_ab; mkdir -p $out
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD:$PYTHONPATH HIPSNAPSHOT_BENCH_DIR=$PWD/bench_tmp
mkdir -p $HIPSNAPSHOT_BENCH_DIR
for i in 1 2; do for ts in 1 0; do for w in 8 1; do
  HIPSNAPSHOT_THREAD_STAGING=$ts timeout -k 10 200 python benchmarks/rank_share/main.py --world $w --steps 10 --warmup 2 \
      --async-iters 3 --restore-iters 1 > $out/w${w}_ts${ts}_$i.json 2>$out/w${w}_ts${ts}_$i.err || { echo FAIL; tail $out/w${w}_ts${ts}_$i.err; exit 1; }
  echo "w=$w ts=$ts $i $(tail -1 $out/w${w}_ts${ts}_$i.json | python -c 'import json,sys; d=json.load(sys.stdin); print(d["take_ms_median"], d["take_ms_min"], d["unblock_ms_median"], d["async_total_ms_median"])')"
done; done; done
for ts in 1 0; do
  HIPSNAPSHOT_THREAD_STAGING=$ts timeout -k 10 300 python bench.py --steps 5 --warmup 2 > $out/bench_ts$ts.json 2> $out/bench_ts$ts.err || { echo FAIL bench; tail $out/bench_ts$ts.err; exit 1; }
  echo "bench ts=$ts $(tail -1 $out/bench_ts$ts.json | cut -c1-200)"
done
