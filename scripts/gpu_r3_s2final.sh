#!/bin/bash
# Session 2, final check: full GPU suite, smoke, headline bench (+ rocprofv3
# kernel/copy stats), the training overlap at seq 512 and 2048.
set -o pipefail
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD HIPSNAPSHOT_BENCH_DIR=$PWD/bench_tmp
O=$PWD/gpurun_out/s2final
mkdir -p $O bench_tmp
TESTS=1 STEPS=20 PROF=1 bash scripts/gpu_check.sh || exit 1
for seq in 512 2048; do
  timeout -k 10 500 python benchmarks/train_overlap/main.py --seq $seq --checkpoints 5 \
      --gap-steps 15 --window-steps 30 --compression hsz1 > $O/ov$seq.json 2> $O/ov$seq.err \
      || { echo OVERLAP_FAIL $seq; tail -20 $O/ov$seq.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/ov$seq.json').read().strip().splitlines()[-1]);print('$seq', {k:d.get(k) for k in ['baseline_step_ms','sync_take_s','cold_async_unblock_ms','async_unblock_ms_each','async_drain_s_each','slowdown_during_drain','train_time_lost_ms','train_time_lost_vs_sync_take','train_time_lost_local_vs_sync_take']})"
done
rm -rf bench_tmp
