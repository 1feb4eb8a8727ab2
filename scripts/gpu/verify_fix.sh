#!/bin/bash
# Round 6: the VMM-backed restore pools.  GPU suite, churn with VMM uncached
# blocks beside hipMalloc'd plain ones, the round-5 trim probe on the fixed
# engine, and a short bench (no regression).
set -o pipefail
O=gpurun_out/r6/fix
mkdir -p $O
export PYTHONUNBUFFERED=1 HSBENCH_DIR=$PWD/bench_tmp
mkdir -p $HSBENCH_DIR
timeout -k 10 150 python scripts/probes/pool_churn_mp.py --mode both --alloc mixed --iters 300 --out $O/churn_mixed.json > $O/churn_mixed.log 2>&1 || { tail -20 $O/churn_mixed.log; exit 1; }
echo "churn_mixed $(tail -1 $O/churn_mixed.log)"
timeout -k 10 240 python scripts/probes/trim_probe_diag.py $O/diag both0 none > $O/diag.log 2>&1 || { tail -20 $O/diag.log; exit 1; }
grep "mode=" $O/diag.log
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests > $O/gputests.log 2>&1 || { grep -E "FAILED|Error|error" $O/gputests.log | tail -20; tail -5 $O/gputests.log; exit 1; }
tail -1 $O/gputests.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -1 $O/bench.json
