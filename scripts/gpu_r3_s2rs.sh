#!/bin/bash
# Session 2: the 8-GPU share at HEAD, solo and with 7 host siblings (rehearsal
# of one rank's host contention on this box's 16-CPU share), 2 runs.
set -o pipefail
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD HIPSNAPSHOT_BENCH_DIR=$PWD/bench_tmp
O=$PWD/gpurun_out/s2rs
mkdir -p $O bench_tmp
for i in 1 2; do
  timeout -k 10 400 python benchmarks/rank_share/main.py --world 8 --steps 10 --warmup 3 --async-iters 3 \
      --restore-iters 2 --host-siblings 7 --sibling-dma-pass 1 > $O/w8_sib7_$i.json 2> $O/w8_sib7_$i.err \
      || { echo RANKSHARE_FAIL; tail -20 $O/w8_sib7_$i.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/w8_sib7_$i.json').read().strip().splitlines()[-1]);print({k:d.get(k) for k in ['take_ms_median','contended_take_ms_median','contended_vs_solo','contended_aggregate_GBps','unblock_ms_median','restore_bitwise_ok']})"
done
rm -rf bench_tmp
