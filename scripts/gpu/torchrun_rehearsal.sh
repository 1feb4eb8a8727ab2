#!/bin/bash
# The driver's multi-GPU launch shape, rehearsed on the one GPU:
#   python -m torch.distributed.run --nnodes=1 --nproc-per-node N
#       --master-addr 127.0.0.1 --master-port P bench.py --gpus N ...
# with gloo (RCCL refuses two ranks on one device).  Every phase runs: FSDP
# takes, async, restore + verify, elastic N -> N/2, HSDP (N >= 4), raw, fresh
# directories, DDP Llama (DDP_LAYERS layers so N replicas fit one card).
#   N=4 DDP_LAYERS=12 OUT=gpurun_out/torchrun ARGS="..."
set -o pipefail
O=${OUT:-gpurun_out/torchrun}
mkdir -p $O
export PYTHONUNBUFFERED=1 HSBENCH_DIR=$PWD/bench_tmp
mkdir -p $HSBENCH_DIR
N=${N:-4}
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N \
    --master-addr 127.0.0.1 --master-port 29631 bench.py --gpus $N --backend gloo \
    --steps 3 --warmup 1 --async-iters 2 --restore-iters 2 --raw-steps 1 --fresh-steps 2 \
    --ddp-steps 0 --ddp-llama-layers ${DDP_LAYERS:-12} --no-numa-bind ${ARGS:-} \
    > $O/torchrun${N}.json 2> $O/torchrun${N}.err \
    || { echo TORCHRUN_FAIL; tail -40 $O/torchrun${N}.err; exit 1; }
grep '^{' $O/torchrun${N}.json | tail -1 | cut -c1-2500
