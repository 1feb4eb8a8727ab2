#!/bin/bash
# Round-2 refresh of the benchmarks not in gpu_bench_all.sh (FSDP nn.Transformer,
# ZeRO-3 OPT, DDP Llama-3-8B, DDP 20 GB with HSZ1).  Each step bounded.
set -o pipefail
mkdir -p gpurun_out/benches
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD:$PYTHONPATH HIPSNAPSHOT_BENCH_DIR=$PWD/bench_tmp
mkdir -p $HIPSNAPSHOT_BENCH_DIR
R=gpurun_out/benches
run() { name=$1; shift; echo "== $name"; timeout -k 10 ${T:-420} "$@" > $R/$name.json 2> $R/$name.err || { echo "FAIL $name"; tail -20 $R/$name.err; exit 1; }; tail -1 $R/$name.json; }
run ddp_20gb_hsz1 python benchmarks/ddp/main.py --repeats 3 --compression hsz1
run fsdp_transformer python benchmarks/fsdp/main.py --torch-save
run zero3_opt python benchmarks/deepspeed_opt/main.py --torch-save
run ddp_llama3_8b python benchmarks/ddp/main.py --model llama3_8b --repeats 3 --torch-save
