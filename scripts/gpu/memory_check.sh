#!/bin/bash
# Round 6: adaptive memory GPU tests, the VMM block cost, the churn probe
# with per-address kind history (malloc, one process: what a re-used address
# was before), and the bench's memory report.
set -o pipefail
O=gpurun_out/r6/mem
mkdir -p $O
export PYTHONUNBUFFERED=1 HSBENCH_DIR=$PWD/bench_tmp
mkdir -p $HSBENCH_DIR
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_memory.py > $O/memtests.log 2>&1 || { grep -E "FAILED|Error" $O/memtests.log | tail -20; tail -30 $O/memtests.log; exit 1; }
tail -1 $O/memtests.log
timeout -k 10 120 python scripts/probes/vmm_cost.py > $O/vmm_cost.json 2> $O/vmm_cost.err || { tail -20 $O/vmm_cost.err; exit 1; }
cat $O/vmm_cost.json
timeout -k 10 150 python scripts/probes/pool_churn_mp.py --mode both --procs 1 --iters 400 --out $O/churn_1p_kinds.json > $O/churn_1p_kinds.log 2>&1 || { tail -20 $O/churn_1p_kinds.log; exit 1; }
tail -1 $O/churn_1p_kinds.log
export HSBENCH_DIR=$PWD/bench_tmp
timeout -k 10 420 python benchmarks/dlrm_uvm/main.py --total-gb 8 --uvm --sync-repeats 6 > $O/dlrm_uvm_repeat.json 2> $O/dlrm_uvm_repeat.err || { tail -20 $O/dlrm_uvm_repeat.err; exit 1; }
tail -1 $O/dlrm_uvm_repeat.json | cut -c1-600
