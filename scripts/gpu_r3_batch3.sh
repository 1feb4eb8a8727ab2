#!/bin/bash
# Round 3 batch 3: the full GPU test suite on the current tree (native drain,
# new freeze layout, MX fp8, 2-D / DLRM GPU tests), then batch 2's probes and
# benchmarks.
set -o pipefail
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD
O=$PWD/gpurun_out/r3b
mkdir -p $O
echo "== GPU tests"
timeout -k 10 900 python -u -m pytest -s tests -m gpu -x -v --timeout 300 --timeout-method thread -k "not fsdp_over_tp_save_and_reshard_gpu" 2>&1 \
    | tee $O/gpu_tests.log | grep --line-buffered -E "PASSED|FAILED|ERROR|Timeout" | awk 'NR % 20 == 0 || /FAIL|ERROR|Timeout/' \
    || { echo GPU_TESTS_FAIL; grep -E "FAIL|Error|assert" $O/gpu_tests.log | head -30; exit 1; }
grep -E "passed|failed" $O/gpu_tests.log | tail -1
bash scripts/gpu_r3_batch2.sh
