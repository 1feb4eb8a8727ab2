#!/bin/bash
# Session 2: drain writers capped at half the CPU share (8 on this box), 16 x
# 64 MiB slots: training overlap at seq 512 and 2048, and bench.py's drain.
set -o pipefail
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD HIPSNAPSHOT_BENCH_DIR=$PWD/bench_tmp
O=$PWD/gpurun_out/s2cap
mkdir -p $O bench_tmp
for seq in 2048 512; do
  timeout -k 10 500 python benchmarks/train_overlap/main.py --seq $seq --checkpoints 5 \
      --gap-steps 15 --window-steps 30 --compression hsz1 > $O/ov$seq.json 2> $O/ov$seq.err \
      || { echo OVERLAP_FAIL $seq; tail -20 $O/ov$seq.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/ov$seq.json').read().strip().splitlines()[-1]);print('$seq', {k:d.get(k) for k in ['baseline_step_ms','cold_async_unblock_ms','async_unblock_ms_each','async_drain_s_each','slowdown_during_drain','train_time_lost_ms','train_time_lost_vs_sync_take','train_time_lost_local_vs_sync_take','cgroup_cpu_in_window']})"
done
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --raw-steps 0 --fresh-steps 0 --ddp-steps 0 \
    --restore-iters 1 --async-iters 3 > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail -20 $O/bench.err; exit 1; }
python -c "import json;d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]);print({k:d.get(k) for k in ['value','time_to_unblock_ms','async_total_ms']})"
rm -rf bench_tmp
