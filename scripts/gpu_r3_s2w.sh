#!/bin/bash
# Session 2, call W: multi-rank regression rehearsal of bench.py at HEAD (gloo
# ranks sharing the one GPU; correctness of the N-rank path, NOT scaling data):
# 8 ranks (no DDP phase: 8 x 20 GB replicas would not fit one GPU), 2 ranks with it.
set -o pipefail
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD HIPSNAPSHOT_BENCH_DIR=$PWD/bench_tmp
O=$PWD/gpurun_out/s2w
mkdir -p $O bench_tmp
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
    --master-port 29811 bench.py --gpus 8 --backend gloo --steps 2 --warmup 1 --async-iters 2 --ddp-steps 0 \
    > $O/n8.json 2> $O/n8.err \
    || { echo N8_FAIL; grep -v -i "gloo\|^\[W\|amdgpu.ids" $O/n8.err | tail -30; exit 1; }
tail -1 $O/n8.json; grep -E "^step|^async|^restore|mismatch|fresh|raw" $O/n8.err | head -12
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29812 bench.py --gpus 2 --backend gloo --steps 2 --warmup 1 --async-iters 2 --ddp-steps 1 \
    > $O/n2.json 2> $O/n2.err \
    || { echo N2_FAIL; grep -v -i "gloo\|^\[W\|amdgpu.ids" $O/n2.err | tail -30; exit 1; }
tail -1 $O/n2.json; grep -E "^step|^async|^restore|mismatch|DDP|fresh|raw" $O/n2.err | head -12
rm -rf bench_tmp
