#!/bin/bash
# rocprofv3 kernel trace + stats of the headline bench on HEAD.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5/prof
export PYTHONUNBUFFERED=1
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r5/prof -o run -- python3 bench.py --steps 3 --warmup 1 --async-iters 2 --raw-steps 0 --fresh-steps 0 --ddp-steps 0 --ddp-llama-steps 0 --elastic-iters 0 > gpurun_out/r5/prof/bench.log 2>&1; rc=$?
find gpurun_out/r5/prof -name "*stats*" | head
tail -1 gpurun_out/r5/prof/bench.log | cut -c1-200
exit $rc
