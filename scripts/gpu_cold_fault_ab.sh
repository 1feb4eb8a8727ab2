#!/bin/bash
# cold-process restore, pinned-block fault-in split over 4 threads vs 1 (alternating)
set -o pipefail
out=gpurun_out/cold_restore; mkdir -p $out
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD:$PYTHONPATH HIPSNAPSHOT_BENCH_DIR=$PWD/bench_tmp
mkdir -p $HIPSNAPSHOT_BENCH_DIR
for i in 1 2; do for t in 4 1; do
HIPSNAPSHOT_PINNED_FAULT_THREADS=$t timeout -k 10 300 python benchmarks/cold_restore/main.py \
    > $out/fault$t.$i.json 2> $out/fault$t.$i.err || { echo COLD_FAIL; tail -30 $out/fault$t.$i.err; exit 1; }
echo "threads=$t run=$i $(python3 -c "import json;d=json.load(open('$out/fault$t.$i.json'));print(d['save']['take_s'], d['restore']['restore_s_each'], d['restore']['restore_bitwise_ok'])")"
done; done
