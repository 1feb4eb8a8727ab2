#!/bin/bash
# Session 2, call H: reproduce the bench.py hang with the drain helper on,
# with the helper's stage markers and a Python stack dump (faulthandler on
# SIGABRT) if it hangs again.
set -o pipefail
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD HIPSNAPSHOT_BENCH_DIR=$PWD/bench_tmp PYTHONFAULTHANDLER=1
O=$PWD/gpurun_out/s2h
mkdir -p $O bench_tmp
HIPSNAPSHOT_DRAIN_PROCESS=1 HIPSNAPSHOT_DRAIN_HELPER_DEBUG=1 HIPSNAPSHOT_DRAIN_HELPER_TIMEOUT_S=60 \
  timeout -s ABRT -k 10 150 python bench.py --steps 2 --warmup 1 --raw-steps 0 --fresh-steps 0 \
  --ddp-steps 0 --restore-iters 1 > $O/bench.json 2> $O/bench.err
rc=$?
echo "bench rc=$rc"
grep -v "^frame" $O/bench.err | tail -60
cat $O/bench.json | tail -1
rm -rf bench_tmp
