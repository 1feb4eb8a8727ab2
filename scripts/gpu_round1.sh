#!/bin/bash
# First GPU call: environment probe, smoke, data-plane microbench, bench.
set -o pipefail
mkdir -p gpurun_out
{
  echo "== env"; nproc; free -g; df -hT /tmp /var/tmp . /dev/shm 2>&1; mount | grep -E " / | /tmp " ; rocm-smi --showproductname 2>&1 | head -20
} > gpurun_out/env.txt 2>&1
export PYTHONUNBUFFERED=1
export PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -50 gpurun_out/smoke.log; exit 1; }
timeout -k 10 300 python benchmarks/microbench.py --dir $PWD/hs_micro_tmp > gpurun_out/micro.jsonl 2> gpurun_out/micro.err || { echo MICRO_FAIL; tail -30 gpurun_out/micro.err; exit 1; }
timeout -k 10 600 python bench.py --steps 3 --warmup 1 > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH_FAIL; tail -40 gpurun_out/bench.err; exit 1; }
cat gpurun_out/env.txt gpurun_out/micro.jsonl gpurun_out/bench.json; tail -20 gpurun_out/bench.err
