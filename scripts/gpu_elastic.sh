#!/bin/bash
# BASELINE config 3 rehearsal on one GPU: FSDP Llama-3-8B saved by 8 gloo
# ranks (sharing the GPU), restored by 4 ranks and by 1 rank, checksums compared.
set -o pipefail
mkdir -p gpurun_out/elastic
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD HSBENCH_DIR=$PWD/bench_tmp
mkdir -p bench_tmp
run() { local n=$1; shift; timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port $((29700 + n)) benchmarks/elastic/main.py --backend gloo "$@"; }
run 8 --phase save > gpurun_out/elastic/save8.json 2> gpurun_out/elastic/save8.err || { echo SAVE_FAIL; grep -v "Gloo\|^\[W" gpurun_out/elastic/save8.err | tail -20; exit 1; }
tail -1 gpurun_out/elastic/save8.json
run 4 --phase restore > gpurun_out/elastic/restore4.json 2> gpurun_out/elastic/restore4.err || { echo R4_FAIL; grep -v "Gloo\|^\[W" gpurun_out/elastic/restore4.err | tail -20; exit 1; }
tail -1 gpurun_out/elastic/restore4.json
run 1 --phase restore > gpurun_out/elastic/restore1.json 2> gpurun_out/elastic/restore1.err || { echo R1_FAIL; grep -v "Gloo\|^\[W" gpurun_out/elastic/restore1.err | tail -20; exit 1; }
tail -1 gpurun_out/elastic/restore1.json
