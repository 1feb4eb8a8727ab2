#!/bin/bash
# Session 2, call M: does the arena size / the bench model stall the helper's
# mapping?  probe with 16 GiB (plain, and nccl+numa+takes), bench.py tiny model.
set -o pipefail
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD HIPSNAPSHOT_BENCH_DIR=$PWD/bench_tmp
O=$PWD/gpurun_out/s2m
mkdir -p $O bench_tmp
i=0
for args in "plain" "nccl numa takes"; do
  i=$((i+1))
  PROBE_GIB=16 timeout -k 10 150 python scripts/helper_ipc_probe.py $args > $O/p$i.json 2> $O/p$i.err
  echo "[16 GiB $args] rc=$?"; grep -E "hsdrain_helper.*(mapp|stall)|did not" $O/p$i.err | tail -4; cat $O/p$i.json
done
HIPSNAPSHOT_DRAIN_PROCESS=1 HIPSNAPSHOT_DRAIN_HELPER_DEBUG=1 HIPSNAPSHOT_DRAIN_HELPER_MAP_TIMEOUT_S=20 \
  timeout -k 10 200 python bench.py --model tiny --steps 2 --warmup 1 --raw-steps 0 --fresh-steps 0 \
  --ddp-steps 0 --restore-iters 1 > $O/bench_tiny.json 2> $O/bench_tiny.err
echo "bench tiny rc=$?"; grep -E "hsdrain_helper.*(mapp)|did not|async" $O/bench_tiny.err | tail -8
rm -rf bench_tmp
