#!/bin/bash
# 8 gloo ranks sharing the one GPU: multi-rank correctness of the GPU path
# with the round-2 engine (plan reuse, background metadata gather, SDMA).
# NOT scaling data (one PCIe link, one GPU).
set -o pipefail
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD HIPSNAPSHOT_BENCH_DIR=$PWD/bench_tmp
mkdir -p bench_tmp gpurun_out/rehearse
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
    --master-port 29811 bench.py --gpus 8 --backend gloo --steps 3 --warmup 1 --async-iters 2 \
    --raw-steps 1 --restore-iters 1 \
    > gpurun_out/rehearse/n8_r2.json 2> gpurun_out/rehearse/n8_r2.err \
    || { echo FAIL; grep -v -i "gloo\|^\[W\|amdgpu.ids" gpurun_out/rehearse/n8_r2.err | tail -30; exit 1; }
tail -1 gpurun_out/rehearse/n8_r2.json; grep -E "^step|^async|^restore|^raw|mismatch" gpurun_out/rehearse/n8_r2.err | head -20
