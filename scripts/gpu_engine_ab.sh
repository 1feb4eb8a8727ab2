#!/bin/bash
# A/B of the bulk D2H engine (blit = hipMemcpyAsync copy kernel, sdma = ROCr
# copy engines): headline bench and the training-overlap benchmark,
# interleaved on one box.  Results: gpurun_out/engine_ab/
set -o pipefail
out=gpurun_out/engine_ab
mkdir -p $out
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD:$PYTHONPATH HIPSNAPSHOT_BENCH_DIR=$PWD/bench_tmp
mkdir -p $HIPSNAPSHOT_BENCH_DIR
for i in $(seq 1 ${N:-2}); do
  for eng in blit sdma; do
    HIPSNAPSHOT_D2H_ENGINE=$eng timeout -k 10 200 python bench.py --steps 6 --warmup 2 \
        > $out/bench_${eng}_$i.json 2> $out/bench_${eng}_$i.err || { echo FAIL bench $eng $i; exit 1; }
    echo "bench $eng $i $(tail -1 $out/bench_${eng}_$i.json)"
    HIPSNAPSHOT_D2H_ENGINE=$eng timeout -k 10 280 python benchmarks/train_overlap/main.py \
        --seq 2048 --compression hsz1 > $out/overlap_${eng}_$i.json 2> $out/overlap_${eng}_$i.err \
        || { echo FAIL overlap $eng $i; tail -20 $out/overlap_${eng}_$i.err; exit 1; }
    echo "overlap $eng $i $(tail -1 $out/overlap_${eng}_$i.json)"
  done
done
