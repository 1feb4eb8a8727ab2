#!/bin/bash
# Session 2, call O: timeline of the 100 GB UVM DLRM save (host-resident tables,
# written in place to /dev/shm): where do its 5 s go.
set -o pipefail
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD HIPSNAPSHOT_BENCH_DIR=$PWD/bench_tmp
O=$PWD/gpurun_out/s2o
mkdir -p $O/tl bench_tmp
HIPSNAPSHOT_TIMELINE=$O/tl/dlrm100 DLRM_RESTORE=0 timeout -k 10 600 python benchmarks/dlrm_uvm/main.py --total-gb 100 --uvm \
    --single-path --work-dir /dev/shm > $O/dlrm_uvm_100gb.json 2> $O/dlrm_uvm_100gb.err \
    || { echo DLRM100_FAIL; tail -20 $O/dlrm_uvm_100gb.err; rm -rf /dev/shm/hs_dlrm; exit 1; }
tail -1 $O/dlrm_uvm_100gb.json
ls -la $O/tl | head
rm -rf /dev/shm/hs_dlrm bench_tmp
