#!/bin/bash
# Round-4 session-3 check: native restore tests, W = 8 share (hsz1 / raw,
# NUMA-bound like a rank), the contended W = 8 share (7 host siblings, CPU-s
# per stored GB), the 1-GPU bench, then the seq-512 drain-writers A/B.
set -o pipefail
out=gpurun_out/s3
mkdir -p $out
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD:$PYTHONPATH HSBENCH_DIR=$PWD/bench_tmp
mkdir -p $HSBENCH_DIR
timeout -k 10 300 python -u -m pytest tests/test_native_restore.py -x -q --timeout 120 \
    --timeout-method thread > $out/pytest_native.log 2>&1 || { tail -40 $out/pytest_native.log; exit 1; }
tail -1 $out/pytest_native.log
for c in hsz1 none; do
  timeout -k 10 240 python benchmarks/rank_share/main.py --world 8 --compression $c \
      > $out/rs8_$c.json 2> $out/rs8_$c.err || { echo RS_FAIL $c; tail -30 $out/rs8_$c.err; exit 1; }
  tail -1 $out/rs8_$c.json | cut -c1-700
done
timeout -k 10 400 python benchmarks/rank_share/main.py --world 8 --host-siblings 7 --steps 6 \
    > $out/rs8_sib7.json 2> $out/rs8_sib7.err || { echo SIB_FAIL; tail -30 $out/rs8_sib7.err; exit 1; }
tail -1 $out/rs8_sib7.json | cut -c1-1500
timeout -k 10 400 python bench.py --steps 5 --warmup 2 > $out/bench.json 2> $out/bench.err \
    || { echo BENCH_FAIL; tail -30 $out/bench.err; exit 1; }
tail -1 $out/bench.json
if [ "${OVERLAP:-1}" = "1" ]; then
KNOB=HIPSNAPSHOT_DRAIN_WRITERS VALS="${WVALS:-3 4 8}" N=${NOV:-2} bash scripts/gpu_overlap_ab.sh
fi
