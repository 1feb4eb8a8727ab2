#!/bin/bash
# N gloo ranks sharing the one GPU, started by bench.py itself (no torchrun):
# every phase of the driver's N-GPU command, incl. DDP Llama (DDP_LAYERS
# layers, so N replicas + DDP buckets fit one card) and the elastic N -> N/2
# restore.  The JSON carries rank_diag / rank_skew for every rank.
#   N=8 DDP_LAYERS=4 OUT=gpurun_out/rehearsal ARGS="..."
set -o pipefail
O=${OUT:-gpurun_out/rehearsal}
mkdir -p $O
export PYTHONUNBUFFERED=1 HSBENCH_DIR=$PWD/bench_tmp
mkdir -p $HSBENCH_DIR
N=${N:-8}
timeout -k 10 1000 python bench.py --gpus $N --backend gloo --steps 2 --warmup 1 \
    --async-iters 2 --restore-iters 2 --raw-steps 1 --fresh-steps 0 --ddp-steps 0 \
    --ddp-llama-layers ${DDP_LAYERS:-4} --no-numa-bind ${ARGS:-} \
    > $O/reh${N}.json 2> $O/reh${N}.err \
    || { echo REH_FAIL; tail -40 $O/reh${N}.err; exit 1; }
tail -1 $O/reh${N}.json | cut -c1-3000
