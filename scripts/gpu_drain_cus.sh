#!/bin/bash
# In-process training overlap vs the async drain's grid cap (HIPSNAPSHOT_DRAIN_CUS).
set -o pipefail
out=gpurun_out/drain_cus
mkdir -p $out
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD:$PYTHONPATH HIPSNAPSHOT_BENCH_DIR=$PWD/bench_tmp
mkdir -p $HIPSNAPSHOT_BENCH_DIR
i=0
for c in ${CUS:-0 32 16 0 32 16}; do
  i=$((i + 1))
  f=$out/run${i}_cus$c
  HIPSNAPSHOT_DRAIN_CUS=$c timeout -k 10 280 python benchmarks/train_overlap/main.py --seq 2048 \
      --compression hsz1 > $f.json 2> $f.err || { echo FAIL $c; tail -20 $f.err; exit 1; }
  echo "cus $c $(tail -1 $f.json)"
done
