#!/bin/bash
# Native restore knob A/B at the W = 8 share (hsz1): one rank_share run per
# setting, restore A/B of one knob inside each run (RESTORE_AB="NAME=v1,v2").
set -o pipefail
out=gpurun_out/restore_knobs
mkdir -p $out
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD:$PYTHONPATH HSBENCH_DIR=$PWD/bench_tmp
mkdir -p $HSBENCH_DIR
i=0
for ab in ${ABS:-HIPSNAPSHOT_NATIVE_RESTORE=1,0 HIPSNAPSHOT_RESTORE_READERS=4,8,12 HIPSNAPSHOT_RESTORE_SLOT_BYTES=4194304,16777216,33554432}; do
  i=$((i+1))
  timeout -k 10 300 python benchmarks/rank_share/main.py --world ${W:-8} --compression ${COMP:-hsz1} \
      --steps 1 --warmup 1 --async-iters 1 --restore-iters ${RI:-5} --ab $ab \
      > $out/ab$i.json 2> $out/ab$i.err || { echo FAIL $ab; tail -20 $out/ab$i.err; exit 1; }
  grep restore_ab $out/ab$i.json; tail -1 $out/ab$i.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["restore_ms_median"], d["native_restore_stats"])'
done
