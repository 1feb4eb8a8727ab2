#!/bin/bash
# Session 2, call I: which process state makes the drain helper's arena
# mapping stall (scripts/helper_ipc_probe.py: no process group / RCCL / gloo).
set -o pipefail
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD HIPSNAPSHOT_BENCH_DIR=$PWD/bench_tmp
O=$PWD/gpurun_out/s2i
mkdir -p $O bench_tmp
for m in plain gloo nccl; do
  timeout -k 10 90 python scripts/helper_ipc_probe.py $m > $O/$m.json 2> $O/$m.err
  echo "$m rc=$?"; grep -E "hsdrain_helper|Error" $O/$m.err | tail -8; cat $O/$m.json
done
cat /proc/sys/kernel/yama/ptrace_scope 2>/dev/null | sed 's/^/ptrace_scope=/'
rm -rf bench_tmp
