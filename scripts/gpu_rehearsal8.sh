#!/bin/bash
# 8 gloo ranks sharing the one GPU, started by bench.py itself (no torchrun):
# every phase of the driver's 8-GPU command, incl. DDP Llama (4 layers, so 8
# replicas + DDP buckets fit one card) and the elastic 8 -> 4 restore.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 HSBENCH_DIR=$PWD/bench_tmp
mkdir -p $HSBENCH_DIR
N=${N:-8}
timeout -k 10 1000 python bench.py --gpus $N --backend gloo --steps 2 --warmup 1 \
    --async-iters 2 --restore-iters 2 --raw-steps 1 --fresh-steps 0 --ddp-steps 0 \
    --ddp-llama-layers ${DDP_LAYERS:-4} --no-numa-bind ${ARGS:-} \
    > gpurun_out/reh${N}.json 2> gpurun_out/reh${N}.err \
    || { echo REH_FAIL; tail -40 gpurun_out/reh${N}.err; exit 1; }
cat gpurun_out/reh${N}.json
