#!/bin/bash
# Session 2, call U: seq-512 training overlap, drain defaults (8 writers, 12 x
# 32 MiB slots) vs 16 writers + 16 x 64 MiB slots (PCIe-bound drain when idle),
# interleaved, twice each.
set -o pipefail
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD HIPSNAPSHOT_BENCH_DIR=$PWD/bench_tmp
O=$PWD/gpurun_out/s2u
mkdir -p $O bench_tmp
for i in 1 2; do
for v in def big; do
  if [ $v = big ]; then E="HIPSNAPSHOT_DRAIN_WRITERS=16 HIPSNAPSHOT_DRAIN_SLOTS=16 HIPSNAPSHOT_DRAIN_SLOT_BYTES=67108864"; else E="HIPSNAPSHOT_X=0"; fi
  env $E timeout -k 10 400 python benchmarks/train_overlap/main.py --seq 512 --checkpoints 5 \
      --gap-steps 15 --window-steps 30 --compression hsz1 > $O/ov512_${v}_$i.json 2> $O/ov512_${v}_$i.err \
      || { echo OVERLAP_FAIL $v; tail -20 $O/ov512_${v}_$i.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/ov512_${v}_$i.json').read().strip().splitlines()[-1]);print('$v $i', {k:d.get(k) for k in ['baseline_step_ms','async_drain_s_each','slowdown_during_drain','train_time_lost_ms','train_time_lost_vs_sync_take','train_time_lost_local_vs_sync_take']})"
done
done
rm -rf bench_tmp
