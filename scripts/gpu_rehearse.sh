#!/bin/bash
# Multi-rank rehearsal on ONE GPU: N ranks share cuda:0 with gloo collectives.
# Exercises the N-rank take/commit/restore path of bench.py (correctness + fixed
# per-step overheads); bandwidth is shared, so these are not scaling numbers.
set -o pipefail
mkdir -p gpurun_out/rehearse gpurun_out/timeline
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD:$PYTHONPATH HIPSNAPSHOT_BENCH_DIR=$PWD/bench_tmp
mkdir -p $HIPSNAPSHOT_BENCH_DIR
port=29731
for n in ${RANKS:-2 4 8}; do
  port=$((port+1))
  HIPSNAPSHOT_TIMELINE=$PWD/gpurun_out/timeline/r$n timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $port bench.py --gpus $n --backend gloo --steps 3 --warmup 1 --async-iters 1 > gpurun_out/rehearse/n$n.json 2> gpurun_out/rehearse/n$n.err || { echo FAIL n=$n; grep -v -i "gloo\|^\[W" gpurun_out/rehearse/n$n.err | tail -30; exit 1; }
  cat gpurun_out/rehearse/n$n.json; grep -E "^step|^async|^restore" gpurun_out/rehearse/n$n.err
  python scripts/timeline_summary.py gpurun_out/timeline/r$n.rank0.take3.json > gpurun_out/rehearse/tl$n.txt 2>&1; head -16 gpurun_out/rehearse/tl$n.txt
done
