#!/bin/bash
# BASELINE config 5 at 70B rank-share scale (train-step overlap), config 4 at
# the W=8 share with host siblings, and the plan-GC A/B of the cold take.
set -o pipefail
R=gpurun_out/r5/g
mkdir -p $R
export PYTHONUNBUFFERED=1 HSBENCH_DIR=$PWD/bench_tmp
mkdir -p $HSBENCH_DIR
run() { name=$1; shift; echo "== $name"; timeout -k 10 ${T:-500} "$@" > $R/$name.json 2> $R/$name.err || { echo "FAIL $name"; grep -v "^frame" $R/$name.err | tail -20; exit 1; }; tail -1 $R/$name.json | cut -c1-1500; }
T=300 run bench_noplangc python bench.py --steps 3 --warmup 1 --async-iters 2 --raw-steps 0 --fresh-steps 0 --ddp-steps 0 --ddp-llama-steps 0 --restore-iters 1 --verify-iters 0 --no-plan-gc
grep -E "warmup|step|async" $R/bench_noplangc.err | head
T=600 run overlap70b_fs python benchmarks/train_overlap/main.py --model llama3_70b --layers 10 --seq 2048 --compression none --checkpoints 2 --gap-steps 10 --window-steps 30
T=600 run overlap70b_s3 python benchmarks/train_overlap/main.py --model llama3_70b --layers 10 --seq 2048 --compression none --storage s3 --checkpoints 2 --gap-steps 10 --window-steps 30
T=600 run dlrm_uvm_w8share python benchmarks/dlrm_uvm/main.py --total-gb 12.5 --uvm --host-siblings 7
rm -rf $HSBENCH_DIR
