#!/bin/bash
# 8 gloo ranks sharing the one GPU (multi-rank correctness of the GPU path,
# NOT scaling data), then the 1-rank headline bench with timelines.
set -o pipefail
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD HIPSNAPSHOT_BENCH_DIR=$PWD/bench_tmp
mkdir -p bench_tmp gpurun_out/rehearse gpurun_out/timeline
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
    --master-port 29811 bench.py --gpus 8 --backend gloo --steps 2 --warmup 1 --async-iters 1 \
    > gpurun_out/rehearse/n8_hsz1.json 2> gpurun_out/rehearse/n8_hsz1.err \
    || { echo FAIL; grep -v -i "gloo\|^\[W\|amdgpu.ids" gpurun_out/rehearse/n8_hsz1.err | tail -30; exit 1; }
cat gpurun_out/rehearse/n8_hsz1.json; grep -E "^step|^async|^restore|mismatch" gpurun_out/rehearse/n8_hsz1.err | head
HIPSNAPSHOT_TIMELINE=$PWD/gpurun_out/timeline/ov timeout -k 10 600 python bench.py --steps 5 --warmup 2 --async-iters 2 \
    > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH_FAIL; tail -30 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json; grep -E "^step|^async|restore" gpurun_out/bench.err
