#!/bin/bash
# Session 2, call P: 100 GB UVM DLRM save through the DMA path (host-resident
# tables copied by SDMA into pinned memory, then written) vs in place, and
# 25 GB in place (does the per-byte rate fall with size?).
set -o pipefail
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD HIPSNAPSHOT_BENCH_DIR=$PWD/bench_tmp
O=$PWD/gpurun_out/s2p
mkdir -p $O bench_tmp
HIPSNAPSHOT_UVM_ASSUME_HOST=0 DLRM_RESTORE=0 timeout -k 10 600 python benchmarks/dlrm_uvm/main.py --total-gb 100 --uvm \
    --single-path --work-dir /dev/shm > $O/dlrm100_dma.json 2> $O/dlrm100_dma.err \
    || { echo DLRM100_FAIL; tail -20 $O/dlrm100_dma.err; rm -rf /dev/shm/hs_dlrm; exit 1; }
tail -1 $O/dlrm100_dma.json
rm -rf /dev/shm/hs_dlrm
DLRM_RESTORE=0 timeout -k 10 600 python benchmarks/dlrm_uvm/main.py --total-gb 25 --uvm \
    --single-path --work-dir /dev/shm > $O/dlrm25_inplace.json 2> $O/dlrm25_inplace.err \
    || { echo DLRM25_FAIL; tail -20 $O/dlrm25_inplace.err; rm -rf /dev/shm/hs_dlrm; exit 1; }
tail -1 $O/dlrm25_inplace.json
rm -rf /dev/shm/hs_dlrm bench_tmp
numactl -H 2>/dev/null | head -5 || true
