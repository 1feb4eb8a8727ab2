#!/bin/bash
# Round 6: which device-memory churn corrupts data across processes on one GPU
# (scripts/probes/pool_churn_mp.py).  One JSON line per configuration.
set -o pipefail
O=gpurun_out/r6/churn
mkdir -p $O
export PYTHONUNBUFFERED=1
run() {  # name, probe args...
  local name=$1; shift
  timeout -k 10 150 python scripts/probes/pool_churn_mp.py "$@" --out $O/$name.json > $O/$name.log 2>&1 || { echo "$name FAILED"; tail -20 $O/$name.log; return 1; }
  echo "$name $(tail -1 $O/$name.log)"
}
run vmm_both --mode both --alloc vmm --iters 300 &&
run malloc_both_1p --mode both --procs 1 --iters 600 &&
run malloc_plain --mode plain --iters 300 &&
run malloc_uc --mode uc --iters 300 &&
run malloc_none --mode none --iters 300 &&
run malloc_both --mode both --iters 300 &&
run vmm_both_8p --mode both --alloc vmm --procs 8 --iters 300
