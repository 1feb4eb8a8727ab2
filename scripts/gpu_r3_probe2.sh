#!/bin/bash
# Round 3: page-cache DMA persistence + threaded throughput; 8-rank async_take
# timeline with the unblock-path spans.
set -o pipefail
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD HIPSNAPSHOT_BENCH_DIR=$PWD/bench_tmp
mkdir -p bench_tmp gpurun_out/r3
timeout -k 10 240 python scripts/pagecache_dma_probe2.py $PWD/bench_tmp \
    > gpurun_out/r3/pagecache_dma2.json 2> gpurun_out/r3/pagecache_dma2.err \
    || { echo "probe2 FAIL"; tail -20 gpurun_out/r3/pagecache_dma2.err; exit 1; }
cat gpurun_out/r3/pagecache_dma2.json
rm -rf gpurun_out/r3/tl8b
HIPSNAPSHOT_TIMELINE=$PWD/gpurun_out/r3/tl8b/t timeout -k 10 600 python -m torch.distributed.run \
    --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29811 bench.py --gpus 8 \
    --backend gloo --steps 1 --warmup 1 --async-iters 4 --raw-steps 0 --fresh-steps 0 \
    --ddp-steps 0 --no-restore-check \
    > gpurun_out/r3/n8b.json 2> gpurun_out/r3/n8b.err \
    || { echo FAIL; grep -v -i "gloo\|^\[W\|amdgpu.ids" gpurun_out/r3/n8b.err | tail -30; exit 1; }
tail -1 gpurun_out/r3/n8b.json; grep -E "^step|^async" gpurun_out/r3/n8b.err | head -20
