#!/bin/bash
# Round 5, first GPU call: RCCL forced-collective tests (+ debug log), the
# headline bench with forced collectives, and the ZeRO-3 save A/B on the
# drain's writer counts.  Each step bounded; stop at the
# first failure.
set -o pipefail
R=gpurun_out/r5/a
mkdir -p $R
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD:$PYTHONPATH HSBENCH_DIR=$PWD/bench_tmp
mkdir -p $HSBENCH_DIR
HSTEST_ARTIFACTS=$R/rccl_forced timeout -k 10 300 python -u -m pytest -x -v --timeout 240 \
    --timeout-method thread tests/test_gpu.py -k "rccl" > $R/rccl_tests.log 2>&1 \
    || { echo "FAIL rccl tests"; tail -60 $R/rccl_tests.log; exit 1; }
tail -4 $R/rccl_tests.log
echo "== bench, forced collectives"
HIPSNAPSHOT_FORCE_COLLECTIVES=1 NCCL_DEBUG=INFO NCCL_DEBUG_SUBSYS=COLL \
    NCCL_DEBUG_FILE=$PWD/$R/bench_forced_rccl.%p.log \
    timeout -k 10 420 python bench.py --steps 5 --warmup 1 > $R/bench_forced.json 2> $R/bench_forced.err \
    || { echo "FAIL bench"; tail -30 $R/bench_forced.err; exit 1; }
tail -1 $R/bench_forced.json | cut -c1-600
run() { name=$1; shift; echo "== $name"; timeout -k 10 ${T:-420} "$@" > $R/$name.json 2> $R/$name.err || { echo "FAIL $name"; tail -20 $R/$name.err; exit 1; }; tail -1 $R/$name.json | cut -c1-400; }
run ds_default python benchmarks/deepspeed_opt/main.py --layers 4 --no-load
HIPSNAPSHOT_TIMELINE=$PWD/$R/tl_ds_default run ds_default_tl python benchmarks/deepspeed_opt/main.py --layers 4 --no-load
HIPSNAPSHOT_DRAIN_BOOST_WRITERS=16 run ds_boost16 python benchmarks/deepspeed_opt/main.py --layers 4 --no-load
HIPSNAPSHOT_DRAIN_WRITERS=16 HIPSNAPSHOT_DRAIN_BOOST_WRITERS=16 run ds_w16 python benchmarks/deepspeed_opt/main.py --layers 4 --no-load
HIPSNAPSHOT_DRAIN_WRITERS=16 HIPSNAPSHOT_DRAIN_BOOST_WRITERS=16 HIPSNAPSHOT_TIMELINE=$PWD/$R/tl_ds_w16 run ds_w16_tl python benchmarks/deepspeed_opt/main.py --layers 4 --no-load
rm -rf $HSBENCH_DIR
