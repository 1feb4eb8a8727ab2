#!/bin/bash
# Round-4 measurement call: fp8 kernels, W=8 rank share (solo, with 7 host
# siblings, and a phase timeline), training overlap trace at seq 512.
set -o pipefail
bash scripts/gpu_fp8.sh || exit 1
out=gpurun_out/rank_share
mkdir -p $out
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD:$PYTHONPATH HSBENCH_DIR=$PWD/bench_tmp
mkdir -p $HSBENCH_DIR
timeout -k 10 300 python benchmarks/rank_share/main.py --world 8 --restore-iters 5 \
    > $out/w8.json 2> $out/w8.err || { echo FAIL w8; tail -20 $out/w8.err; exit 1; }
tail -1 $out/w8.json
HIPSNAPSHOT_TIMELINE=$PWD/$out/tl8 timeout -k 10 300 python benchmarks/rank_share/main.py --world 8 \
    --steps 3 --warmup 2 --async-iters 1 --restore-iters 3 > $out/tl8.json 2> $out/tl8.err \
    || { echo FAIL tl; tail -20 $out/tl8.err; exit 1; }
for f in $out/tl8.rank0.restore*.json $out/tl8.rank0.take*.json; do python3 scripts/timeline_summary.py $f > ${f%.json}.txt; done
tail -30 $out/tl8.rank0.restore2.txt
timeout -k 10 400 python benchmarks/rank_share/main.py --world 8 --host-siblings 7 --restore-iters 3 \
    > $out/w8_sib7.json 2> $out/w8_sib7.err || { echo FAIL sib; tail -20 $out/w8_sib7.err; exit 1; }
tail -1 $out/w8_sib7.json
bash scripts/gpu_overlap_trace.sh
