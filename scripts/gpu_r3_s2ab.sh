#!/bin/bash
# Session 2: what slows a launch-bound (seq 512) training step while a drain
# runs -- default, no blob checksums, hash stream at default priority,
# 2 drain slots in flight (half the PCIe rate).
set -o pipefail
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD HIPSNAPSHOT_BENCH_DIR=$PWD/bench_tmp
O=$PWD/gpurun_out/s2ab
mkdir -p $O bench_tmp
for v in default nosum hashlow slots2; do
  case $v in
    default) E="HIPSNAPSHOT_X=0";;
    nosum) E="HIPSNAPSHOT_CHECKSUM=0";;
    hashlow) E="HIPSNAPSHOT_DRAIN_HASH_HIGH_PRIORITY=0";;
    slots2) E="HIPSNAPSHOT_DRAIN_SLOTS=2";;
  esac
  env $E timeout -k 10 400 python benchmarks/train_overlap/main.py --seq 512 --checkpoints 5 \
      --gap-steps 15 --window-steps 30 --compression hsz1 > $O/ov512_$v.json 2> $O/ov512_$v.err \
      || { echo OVERLAP_FAIL $v; tail -20 $O/ov512_$v.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/ov512_$v.json').read().strip().splitlines()[-1]);print('$v', {k:d.get(k) for k in ['baseline_step_ms','async_drain_s_each','slowdown_during_drain','slowdown_local_median_each','train_time_lost_vs_sync_take','train_time_lost_local_vs_sync_take']})"
done
rm -rf bench_tmp
