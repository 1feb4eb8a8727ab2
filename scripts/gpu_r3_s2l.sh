#!/bin/bash
# Session 2, call L: which part of bench.py's process state stalls the drain
# helper's IPC mapping: NUMA CPU binding, prior blocking takes, both.
set -o pipefail
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD HIPSNAPSHOT_BENCH_DIR=$PWD/bench_tmp
O=$PWD/gpurun_out/s2l
mkdir -p $O bench_tmp
i=0
for args in "plain" "plain numa" "plain takes" "nccl numa takes"; do
  i=$((i+1))
  timeout -k 10 120 python scripts/helper_ipc_probe.py $args > $O/p$i.json 2> $O/p$i.err
  echo "[$args] rc=$?"; grep -E "hsdrain_helper.*(mapp|stall)|did not|bound" $O/p$i.err | tail -4; cat $O/p$i.json
done
rm -rf bench_tmp
