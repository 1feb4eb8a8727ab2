#!/bin/bash
# Is the training slowdown during an async drain CPU contention? Overlap
# benchmark (hsz1) with the default I/O workers, fewer workers, and niced
# workers (HIPSNAPSHOT_IO_NICE), interleaved twice.
set -o pipefail
out=gpurun_out/overlap_cpu
mkdir -p $out
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD:$PYTHONPATH HIPSNAPSHOT_BENCH_DIR=$PWD/bench_tmp
mkdir -p $HIPSNAPSHOT_BENCH_DIR
nproc; python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)))"; cat /sys/fs/cgroup/cpu.max 2>/dev/null || true
run() {  # name env...
  local name=$1; shift
  env "$@" timeout -k 10 600 python benchmarks/train_overlap/main.py --seq 512 \
      --baseline-steps 10 ${ARGS:-} > $out/$name.json 2> $out/$name.err \
      || { echo OVERLAP_FAIL $name; grep -v "^frame" $out/$name.err | tail -30; return 1; }
  echo "$name $(tail -1 $out/$name.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ["baseline_step_ms","async_drain_s","steps_during_drain","step_ms_during_drain_mean","slowdown_during_drain"]})')"
}
for r in 1 2; do
  run default_r$r HIPSNAPSHOT_IO_NICE=0 || exit 1
  run io4_r$r HIPSNAPSHOT_IO_THREADS=4 || exit 1
  run nice10_r$r HIPSNAPSHOT_IO_NICE=10 || exit 1
  run nice19_r$r HIPSNAPSHOT_IO_NICE=19 || exit 1
done
