#!/bin/bash
# Session 2, last call: full GPU suite, smoke, bench; then one counter pass
# (TCC_EA0_RDREQ + TCC_EA0_RDREQ_32B) over the fp8 kernels to check how many
# bytes a read request carries (FETCH_SIZE assumes 64 B for non-32-B ones).
set -o pipefail
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD
REPO=$PWD
TESTS=1 STEPS=5 bash scripts/gpu_check.sh || exit 1
mkdir -p gpurun_out/s2last
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --kernel-trace --stats --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum \
    --kernel-include-regex "hs_" --output-format csv -d $REPO/gpurun_out/s2last/rdreq -o pmc \
    -- python3 $REPO/scripts/fp8_kernels_bench.py mx_e8m0 none \
    > $REPO/gpurun_out/s2last/rdreq.log 2>&1 || { echo PMC_FAIL; tail -20 $REPO/gpurun_out/s2last/rdreq.log; exit 0; }
find $REPO/gpurun_out/s2last -name "*counter_collection.csv"
