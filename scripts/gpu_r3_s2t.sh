#!/bin/bash
# Session 2, call T: the async drain of the 16 GB Llama-3-8B state with an
# idle trainer (bench.py's async_total_ms, ~380 ms = 42 GB/s raw): writer /
# slot sweep with per-phase stats.
set -o pipefail
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD HIPSNAPSHOT_BENCH_DIR=$PWD/bench_tmp
O=$PWD/gpurun_out/s2t
mkdir -p $O bench_tmp
for cfg in "8 12 33554432" "16 12 33554432" "8 24 33554432" "16 24 33554432" "16 16 67108864"; do
  set -- $cfg
  tag=w$1_s$2_b$(( $3 >> 20 ))
  HIPSNAPSHOT_DRAIN_WRITERS=$1 HIPSNAPSHOT_DRAIN_SLOTS=$2 HIPSNAPSHOT_DRAIN_SLOT_BYTES=$3 \
    timeout -k 10 300 python bench.py --steps 1 --warmup 1 --raw-steps 0 --fresh-steps 0 --ddp-steps 0 \
    --restore-iters 1 --async-iters 4 > $O/$tag.json 2> $O/$tag.err \
    || { echo BENCH_FAIL $tag; tail -20 $O/$tag.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]);st=d.get('async_drain_stats') or {};print('$tag', d['async_total_ms'], [round(x) for x in [0]], {k:st.get(k) for k in ['wall','slot_wait','sdma_wait','pwrite','sdma_submit','hash_collect']})"
done
rm -rf bench_tmp
