#!/bin/bash
# Session 2, call N: bench.py (Llama-3-8B) with the drain helper: does a
# runtime call in the trainer while the helper maps (DRAIN_HELPER_POKE)
# unstall the mapping?  Then without poking, with the arena kept OFF.
set -o pipefail
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD HIPSNAPSHOT_BENCH_DIR=$PWD/bench_tmp
O=$PWD/gpurun_out/s2n
mkdir -p $O bench_tmp
for v in poke nokeep; do
  if [ $v = poke ]; then E="HIPSNAPSHOT_DRAIN_HELPER_POKE=1"; else E="HIPSNAPSHOT_HBM_ARENA_KEEP=0"; fi
  env $E HIPSNAPSHOT_DRAIN_PROCESS=1 HIPSNAPSHOT_DRAIN_HELPER_DEBUG=1 HIPSNAPSHOT_DRAIN_HELPER_MAP_TIMEOUT_S=20 \
    timeout -k 10 200 python bench.py --steps 2 --warmup 1 --raw-steps 0 --fresh-steps 0 \
    --ddp-steps 0 --restore-iters 1 > $O/bench_$v.json 2> $O/bench_$v.err
  echo "[$v] rc=$?"; grep -E "hsdrain_helper.*(mapp)|did not|async" $O/bench_$v.err | tail -8
done
rm -rf bench_tmp
