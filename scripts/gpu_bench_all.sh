#!/bin/bash
# All BASELINE configs that fit one MI355X. Each step bounded; stop at first failure.
set -o pipefail
mkdir -p gpurun_out/benches
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD:$PYTHONPATH HSBENCH_DIR=$PWD/bench_tmp
mkdir -p $HSBENCH_DIR
R=gpurun_out/benches
run() { name=$1; shift; echo "== $name"; timeout -k 10 ${T:-420} "$@" > $R/$name.json 2> $R/$name.err || { echo "FAIL $name"; tail -20 $R/$name.err; exit 1; }; cat $R/$name.json; }
run ddp_20gb python benchmarks/ddp/main.py --repeats 3 --torch-save
run load_tensor python benchmarks/load_tensor/main.py
run dlrm_uvm python benchmarks/dlrm_uvm/main.py --total-gb 8 --uvm
run dlrm_hbm python benchmarks/dlrm_uvm/main.py --total-gb 8
run async_s3 python benchmarks/async_s3/main.py --model llama3_8b --layers 8
run bench_fsync python bench.py --steps 2 --warmup 1 --async-iters 1 --fsync --no-restore-check
run bench_direct python bench.py --steps 2 --warmup 1 --async-iters 0 --direct-io --no-restore-check
