#!/bin/bash
# W-rank share restore A/B of one knob (interleaved in one process):
# KNOB=NAME VALS=v1,v2 bash scripts/gpu_restore_ab.sh
set -o pipefail
out=gpurun_out/restore_ab
mkdir -p $out
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD:$PYTHONPATH HSBENCH_DIR=$PWD/bench_tmp
mkdir -p $HSBENCH_DIR
for kv in ${ABS:-HIPSNAPSHOT_STAGE_THREADS=4,8}; do
  n=${kv%%=*}
  timeout -k 10 300 python benchmarks/rank_share/main.py --world ${W:-8} --steps 4 --warmup 2 \
      --async-iters 1 --restore-iters ${RI:-6} --ab $kv > $out/$n.json 2> $out/$n.err \
      || { echo FAIL $n; tail -20 $out/$n.err; exit 1; }
  grep restore_ab $out/$n.json
done
