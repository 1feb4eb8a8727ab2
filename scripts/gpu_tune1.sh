#!/bin/bash
# NUMA binding and restore-pipeline knobs, one short bench per variant.
set -o pipefail
mkdir -p gpurun_out/tune
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD:$PYTHONPATH HIPSNAPSHOT_BENCH_DIR=$PWD/bench_tmp
mkdir -p $HIPSNAPSHOT_BENCH_DIR
{ lscpu | head -30; cat /sys/devices/system/node/node*/cpulist; python -c "import os;print('allowed',sorted(os.sched_getaffinity(0)))"; } > gpurun_out/tune/topo.txt 2>&1
run() {  # name, env..., -- args
  local name=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 3 --warmup 1 --async-iters 2 ${EXTRA:-} \
      > gpurun_out/tune/$name.json 2> gpurun_out/tune/$name.err || { echo "FAIL $name"; tail -20 gpurun_out/tune/$name.err; return 1; }
  tail -1 gpurun_out/tune/$name.json | python -c "import json,sys;d=json.loads(sys.stdin.read());print('$name', d['value'], d['ms_per_step'], d['restore_GBps'], d['time_to_unblock_ms'])"; grep -E '^async' gpurun_out/tune/$name.err | tr '\n' ' '; echo
}
run base X=1 && grep numa gpurun_out/tune/base.err &&
EXTRA=--no-numa-bind run nobind X=1 && \
run io32 HIPSNAPSHOT_IO_THREADS=32 && \
run inflight16 HIPSNAPSHOT_READ_INFLIGHT=16 && \
run consume8 HIPSNAPSHOT_STAGE_THREADS=8 && \
run split4 HIPSNAPSHOT_IO_READ_SPLIT_BYTES=4194304
