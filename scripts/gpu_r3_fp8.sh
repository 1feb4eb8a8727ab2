#!/bin/bash
# Round 3: new GPU tests (MX fp8 numerics, DLRM resharding matrix, FSDP2 x TP,
# async live-tensor race), then the fp8 kernels alone: host-timed, rocprofv3
# kernel stats, and FETCH_SIZE / WRITE_SIZE counter passes.
set -o pipefail
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD
REPO=$PWD
mkdir -p gpurun_out/r3/fp8
timeout -k 10 700 python -u -m pytest -s tests/test_dlrm_resharding.py tests/test_dtensor_2d.py tests/test_gpu.py \
    -m gpu -x -v --timeout 300 --timeout-method thread \
    -k "resharding or fsdp_over_tp or unfrozen or mx8 or fp8" 2>&1 | tee gpurun_out/r3/newgpu.log | grep --line-buffered -E "dlrm case|PASS|FAIL|Timeout|Thread|File"  \
    || { echo TESTS_FAIL; grep -E "FAIL|Error|assert" gpurun_out/r3/newgpu.log | head -30; exit 1; }
tail -2 gpurun_out/r3/newgpu.log
timeout -k 10 120 python scripts/fp8_kernels_bench.py > gpurun_out/r3/fp8/host_timed.jsonl 2>&1 \
    || { echo BENCH_FAIL; tail gpurun_out/r3/fp8/host_timed.jsonl; exit 1; }
cat gpurun_out/r3/fp8/host_timed.jsonl
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats --kernel-include-regex "hs_" --output-format csv \
    -d $REPO/gpurun_out/r3/fp8/trace -o fp8 -- python3 $REPO/scripts/fp8_kernels_bench.py \
    > $REPO/gpurun_out/r3/fp8/trace.log 2>&1 || { echo TRACE_FAIL; tail -20 $REPO/gpurun_out/r3/fp8/trace.log; exit 1; }
for pass in FETCH_SIZE WRITE_SIZE; do
  tag=$(echo $pass | tr 'A-Z' 'a-z')
  timeout -s KILL 120 rocprofv3 --kernel-trace --stats --pmc $pass --kernel-include-regex "hs_" \
      --output-format csv -d $REPO/gpurun_out/r3/fp8/pmc_$tag -o pmc -- python3 $REPO/scripts/fp8_kernels_bench.py mx_e8m0 none hadamard32 \
      > $REPO/gpurun_out/r3/fp8/pmc_$tag.log 2>&1 || { echo PMC_FAIL $tag; tail -20 $REPO/gpurun_out/r3/fp8/pmc_$tag.log; exit 1; }
done
find $REPO/gpurun_out/r3/fp8 -name "*.csv" | head -20
