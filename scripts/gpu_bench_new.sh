#!/bin/bash
# Benchmarks added after the first sweep (FSDP nn.Transformer, ZeRO-3 OPT, DDP Llama-3-8B).
set -o pipefail
mkdir -p gpurun_out/benches
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD:$PYTHONPATH HIPSNAPSHOT_BENCH_DIR=$PWD/bench_tmp
mkdir -p $HIPSNAPSHOT_BENCH_DIR
R=gpurun_out/benches
run() { name=$1; shift; echo "== $name"; timeout -k 10 ${T:-420} "$@" > $R/$name.json 2> $R/$name.err || { echo "FAIL $name"; tail -20 $R/$name.err; exit 1; }; cat $R/$name.json; grep -vi gloo $R/$name.err | tail -6; }
run fsdp_transformer python benchmarks/fsdp/main.py --torch-save
run zero3_opt python benchmarks/deepspeed_opt/main.py --torch-save
run ddp_llama3_8b python benchmarks/ddp/main.py --model llama3_8b --repeats 3 --torch-save
echo "== bench timeline"
HIPSNAPSHOT_TIMELINE=$PWD/gpurun_out/timeline/tl timeout -k 10 400 python bench.py --steps 3 --warmup 1 --async-iters 1 > gpurun_out/bench_tl.json 2> gpurun_out/bench_tl.err || { echo FAIL bench_tl; tail -20 gpurun_out/bench_tl.err; exit 1; }
cat gpurun_out/bench_tl.json
python scripts/timeline_summary.py gpurun_out/timeline/tl.rank0.take2.json gpurun_out/timeline/tl.rank0.take3.json gpurun_out/timeline/tl.rank0.restore0.json > gpurun_out/timeline_summary.txt 2>&1; cat gpurun_out/timeline_summary.txt
