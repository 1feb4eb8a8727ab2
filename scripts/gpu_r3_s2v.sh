#!/bin/bash
# Session 2, call V: BASELINE config 5's storage path for its model size: one
# rank's share of Llama-3-70B FSDP at 8 GPUs (17.6 GB) async_take'n to the fake
# S3 server (own process) and restored, bitwise.
set -o pipefail
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD HIPSNAPSHOT_BENCH_DIR=$PWD/bench_tmp
O=$PWD/gpurun_out/s2v
mkdir -p $O bench_tmp
timeout -k 10 600 python benchmarks/async_s3/main.py --model llama3_70b --share-of 8 --iters 2 \
    > $O/s3_70b_share8.json 2> $O/s3_70b_share8.err \
    || { echo S3_FAIL; tail -20 $O/s3_70b_share8.err; exit 1; }
grep -E "async_take|restore" $O/s3_70b_share8.err | tail -6
tail -1 $O/s3_70b_share8.json
rm -rf bench_tmp
