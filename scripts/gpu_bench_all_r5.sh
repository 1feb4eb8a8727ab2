#!/bin/bash
# Every single-GPU benchmark on HEAD, then the regression guard
# (scripts/check_thresholds.py, floors in scripts/bench_thresholds.json).
set -o pipefail
R=gpurun_out/benches_r5
mkdir -p $R
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD:$PYTHONPATH HSBENCH_DIR=$PWD/bench_tmp
mkdir -p $HSBENCH_DIR
run() { name=$1; shift; echo "== $name"; timeout -k 10 ${T:-420} "$@" > $R/$name.json 2> $R/$name.err || { echo "FAIL $name"; tail -20 $R/$name.err; exit 1; }; tail -1 $R/$name.json | cut -c1-700; }
run bench python bench.py --steps 5 --warmup 2
run ddp_20gb python benchmarks/ddp/main.py --repeats 3
run fsdp python benchmarks/fsdp/main.py
run load_tensor python benchmarks/load_tensor/main.py
run dlrm_uvm python benchmarks/dlrm_uvm/main.py --total-gb 8 --uvm
run dlrm_hbm python benchmarks/dlrm_uvm/main.py --total-gb 8
run deepspeed_opt python benchmarks/deepspeed_opt/main.py --layers 4
run cold_restore python benchmarks/cold_restore/main.py
run resnet_ddp python benchmarks/resnet_ddp/main.py
run share70b python benchmarks/rank_share/main.py --model llama3_70b --world 8 --steps 3 --warmup 1 --async-iters 2 --restore-iters 3
rm -rf $HSBENCH_DIR
python scripts/check_thresholds.py $R
