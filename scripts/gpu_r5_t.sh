#!/bin/bash
# One rank's W = 8 share on HEAD: solo, then with 7 host siblings (buffered writes).
set -o pipefail
mkdir -p gpurun_out/r5/t
export PYTHONUNBUFFERED=1 HSBENCH_DIR=$PWD/bench_tmp HSBENCH_SIBLING_DIR=/dev/shm/hs_sib
mkdir -p $HSBENCH_DIR
timeout -k 10 400 python benchmarks/rank_share/main.py --world 8 --steps 6 --warmup 2 --async-iters 2 --restore-iters 2 > gpurun_out/r5/t/solo.json 2> gpurun_out/r5/t/solo.err || { tail -20 gpurun_out/r5/t/solo.err; exit 1; }
tail -1 gpurun_out/r5/t/solo.json | cut -c1-700
timeout -k 10 400 python benchmarks/rank_share/main.py --world 8 --host-siblings 7 --steps 6 --warmup 2 --async-iters 2 --restore-iters 2 > gpurun_out/r5/t/sib7.json 2> gpurun_out/r5/t/sib7.err || { tail -20 gpurun_out/r5/t/sib7.err; rm -rf /dev/shm/hs_sib; exit 1; }
rm -rf /dev/shm/hs_sib
tail -1 gpurun_out/r5/t/sib7.json | cut -c1-900
