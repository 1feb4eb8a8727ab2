#!/bin/bash
# One rank's full share of BASELINE configs 4 and 5 at 8 GPUs, on one GPU:
#   config 5: Llama-3-70B FSDP over 8 ranks -> 17.6 GB of bf16 shards per rank
#             (take, async_take unblock, restore; benchmarks/rank_share)
#   config 4: DLRM with 100 GB of UVM embedding tables over 8 ranks -> 12.5 GB
#             of managed-memory tables per rank (benchmarks/dlrm_uvm)
set -o pipefail
out=gpurun_out/configs_share
mkdir -p $out
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD:$PYTHONPATH HIPSNAPSHOT_BENCH_DIR=$PWD/bench_tmp
mkdir -p $HIPSNAPSHOT_BENCH_DIR
timeout -k 10 400 python benchmarks/rank_share/main.py --model llama3_70b --world 8 \
    --steps 3 --warmup 1 --async-iters 3 --restore-iters 2 \
    > $out/llama70b_w8_hsz1.json 2> $out/llama70b_w8_hsz1.err \
    || { echo FAIL 70b; tail -20 $out/llama70b_w8_hsz1.err; exit 1; }
cat $out/llama70b_w8_hsz1.json
rm -rf $HIPSNAPSHOT_BENCH_DIR/*
timeout -k 10 400 python benchmarks/dlrm_uvm/main.py --total-gb 12.5 --uvm \
    > $out/dlrm_uvm_12p5gb.json 2> $out/dlrm_uvm_12p5gb.err \
    || { echo FAIL dlrm; tail -20 $out/dlrm_uvm_12p5gb.err; exit 1; }
cat $out/dlrm_uvm_12p5gb.json
