#!/bin/bash
# rank-share take with the default GIL switch interval (5 ms) vs shorter ones
set -o pipefail
out=gpurun_out/switch_ab; mkdir -p $out
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD:$PYTHONPATH HIPSNAPSHOT_BENCH_DIR=$PWD/bench_tmp
mkdir -p $HIPSNAPSHOT_BENCH_DIR
for i in 1 2; do for si in 0 0.0005 0.0001; do for w in 8 1; do
  timeout -k 10 200 python benchmarks/rank_share/main.py --world $w --steps 10 --warmup 2 --async-iters 1 --restore-iters 1 \
      --switch-interval $si > $out/w${w}_si${si}_$i.json 2>/dev/null || { echo FAIL; exit 1; }
  echo "w=$w si=$si $i $(tail -1 $out/w${w}_si${si}_$i.json | python -c 'import json,sys; d=json.load(sys.stdin); print(d["take_ms_median"], d["take_ms_min"], d["unblock_ms_median"], d["restore_ms_median"])')"
done; done; done
