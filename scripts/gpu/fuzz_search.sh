#!/bin/bash
# Wide seed search of every randomised GPU test (tests/test_*random*.py,
# test_gpu_fuzz.py, flaky S3): the default counts times ~10-25.
#   OUT=gpurun_out/r6/fuzz_wide
set -o pipefail
O=${OUT:-gpurun_out/r6/fuzz_wide}
mkdir -p $O
export PYTHONUNBUFFERED=1
run() {
  local name=$1; shift
  echo "== $name"
  timeout -k 10 ${T:-400} "$@" > $O/$name.log 2>&1 || { echo "FAIL $name"; grep -E "^E |FAILED" $O/$name.log | head -20; exit 1; }
  tail -1 $O/$name.log
}
P="python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread"
HS_E2E_GPU_SEEDS=600 run e2e $P tests/test_e2e_random.py
HS_ASYNC_GPU_SEEDS=100 run async $P tests/test_async_random.py
HS_QUANT_SEEDS=400 run quant $P tests/test_quant_random.py
HS_UVM_SEEDS=150 run uvm $P tests/test_uvm_random.py
HS_CORRUPT_SEEDS=300 run corrupt $P tests/test_corruption_random.py
HS_RESUME_SEEDS=200 run resume $P tests/test_resume_random.py
HS_FLAKY_SEEDS=12 run flaky_s3 $P tests/test_storage_plugins.py
run kernels $P tests/test_gpu_fuzz.py
