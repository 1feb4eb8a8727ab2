#!/bin/bash
# W = 8 share with 7 host siblings: buffered writes vs O_DIRECT (no CPU copy
# into the page cache), CPU-s per stored GB and take time of each
set -o pipefail
out=gpurun_out/rank_share_direct
mkdir -p $out
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD:$PYTHONPATH HSBENCH_DIR=$PWD/bench_tmp
mkdir -p $HSBENCH_DIR
for mode in buffered direct buffered direct; do
  if [ $mode = direct ]; then export HIPSNAPSHOT_FS_DIRECT_IO=1; else unset HIPSNAPSHOT_FS_DIRECT_IO; fi
  timeout -k 10 300 python benchmarks/rank_share/main.py --world 8 --host-siblings 7 --steps 6 --warmup 2 \
      --async-iters 2 --restore-iters 2 > $out/sib7_$mode.json 2> $out/sib7_$mode.err \
      || { echo FAIL $mode; tail -20 $out/sib7_$mode.err; exit 1; }
  cp $out/sib7_$mode.json $out/sib7_${mode}_$(date +%s).json
  python3 -c "import json,sys; d=json.loads(open('$out/sib7_$mode.json').read().strip().splitlines()[-1]); print('$mode', {k: d[k] for k in d if any(s in k for s in ('take_ms','cpu_s','sibling_host','restore_ms','GBps'))})"
done
