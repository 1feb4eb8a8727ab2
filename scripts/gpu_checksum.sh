#!/bin/bash
# hs64 checksums on the GPU: kernel/verify tests, then the headline bench with
# checksums on and off, interleaved.  Results: gpurun_out/cksum/
set -o pipefail
out=gpurun_out/cksum
mkdir -p $out
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD:$PYTHONPATH HIPSNAPSHOT_BENCH_DIR=$PWD/bench_tmp
mkdir -p $HIPSNAPSHOT_BENCH_DIR
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -v --timeout 120 --timeout-method thread \
    -k "hash or checksum" > $out/tests.log 2>&1 || { echo FAIL tests; tail -30 $out/tests.log; exit 1; }
tail -3 $out/tests.log
for i in $(seq 1 ${N:-2}); do
  for ck in 1 0; do
    HIPSNAPSHOT_CHECKSUM=$ck timeout -k 10 240 python bench.py --steps 5 --warmup 2 \
        > $out/bench_ck${ck}_$i.json 2> $out/bench_ck${ck}_$i.err || { echo FAIL bench $ck $i; tail -20 $out/bench_ck${ck}_$i.err; exit 1; }
    echo "bench ck=$ck $i $(tail -1 $out/bench_ck${ck}_$i.json)"
  done
done
