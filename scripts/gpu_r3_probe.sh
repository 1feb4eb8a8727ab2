#!/bin/bash
# Round 3: (1) SDMA straight into mmap'd page-cache pages (one host DRAM
# crossing) vs pinned + pwrite; (2) 8 gloo ranks sharing the one GPU with a
# timeline of every async_take (span breakdown of time-to-unblock).
set -o pipefail
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD HIPSNAPSHOT_BENCH_DIR=$PWD/bench_tmp
mkdir -p bench_tmp gpurun_out/r3
timeout -k 10 120 python scripts/pagecache_dma_probe.py $PWD/bench_tmp \
    > gpurun_out/r3/pagecache_dma.json 2> gpurun_out/r3/pagecache_dma.err \
    || { echo "probe FAIL"; tail -20 gpurun_out/r3/pagecache_dma.err; }
cat gpurun_out/r3/pagecache_dma.json
HIPSNAPSHOT_TIMELINE=$PWD/gpurun_out/r3/tl8/t timeout -k 10 600 python -m torch.distributed.run \
    --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29811 bench.py --gpus 8 \
    --backend gloo --steps 2 --warmup 1 --async-iters 4 --raw-steps 0 --fresh-steps 0 \
    --ddp-steps 0 --restore-iters 1 \
    > gpurun_out/r3/n8.json 2> gpurun_out/r3/n8.err \
    || { echo FAIL; grep -v -i "gloo\|^\[W\|amdgpu.ids" gpurun_out/r3/n8.err | tail -30; exit 1; }
tail -1 gpurun_out/r3/n8.json; grep -E "^step|^async|^restore|mismatch" gpurun_out/r3/n8.err | head -20
