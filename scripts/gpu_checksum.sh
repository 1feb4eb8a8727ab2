#!/bin/bash
# hs64 checksums on the GPU: kernel/verify tests, then the headline bench
# (hsz1) and a raw-blob bench with checksums on and off, interleaved.
# Results: gpurun_out/cksum/
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
    echo "hsz1 ck=$ck $i $(tail -1 $out/bench_ck${ck}_$i.json | python -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"], d["raw_GBps"], d["time_to_unblock_ms"], d["restore_GBps"])')"
    HIPSNAPSHOT_CHECKSUM=$ck timeout -k 10 240 python bench.py --steps 5 --warmup 2 --compression none \
        --restore-iters 1 > $out/raw_ck${ck}_$i.json 2> $out/raw_ck${ck}_$i.err || { echo FAIL raw $ck $i; tail -20 $out/raw_ck${ck}_$i.err; exit 1; }
    echo "raw ck=$ck $i $(tail -1 $out/raw_ck${ck}_$i.json | python -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"], d["time_to_unblock_ms"])')"
  done
done
