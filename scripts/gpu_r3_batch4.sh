#!/bin/bash
# Round 3 batch 4: Hadamard kernel numerics + speed; the 2-D DTensor GPU test;
# training overlap with back-to-back async checkpoints (native raw drain vs
# Python drain vs encoded drain); rank share W=8 with host siblings sized like
# an 8-rank job (with and without the DMA write pass).
set -o pipefail
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD HIPSNAPSHOT_BENCH_DIR=$PWD/bench_tmp
REPO=$PWD
O=$REPO/gpurun_out/r3c
mkdir -p $O/fp8 bench_tmp
echo "== hadamard + 2-D tests"
timeout -k 10 400 python -u -m pytest -s tests/test_gpu.py tests/test_dtensor_2d.py -m gpu -x -v --timeout 300 \
    --timeout-method thread -k "hadamard or fsdp_over_tp" > $O/tests.log 2>&1 \
    || { echo TESTS_FAIL; grep -E "FAIL|Error|assert" $O/tests.log | head -30; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -1
echo "== fp8 kernels"
timeout -k 10 120 python scripts/fp8_kernels_bench.py > $O/fp8/host_timed.jsonl 2>&1 || { echo BENCH_FAIL; tail $O/fp8/host_timed.jsonl; exit 1; }
cat $O/fp8/host_timed.jsonl
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats --kernel-include-regex "hs_" --output-format csv \
    -d $O/fp8/trace -o fp8 -- python3 $REPO/scripts/fp8_kernels_bench.py \
    > $O/fp8/trace.log 2>&1 || { echo TRACE_FAIL; tail -20 $O/fp8/trace.log; exit 1; }
cd $REPO
for mode in native python encoded; do
  echo "== train_overlap $mode"
  case $mode in
    native) envs="";;
    python) envs="HIPSNAPSHOT_NATIVE_DRAIN=0";;
    encoded) envs="HIPSNAPSHOT_ASYNC_DEVICE_CODEC=same";;
  esac
  env $envs timeout -k 10 420 python benchmarks/train_overlap/main.py --seq 512 --checkpoints 5 \
      --window-steps 30 --compression hsz1 > $O/overlap_$mode.json 2> $O/overlap_$mode.err \
      || { echo OVERLAP_FAIL $mode; tail -20 $O/overlap_$mode.err; exit 1; }
  tail -1 $O/overlap_$mode.json
done
for dp in 0 1; do
  echo "== rank share W=8 + 7 host siblings, dma pass $dp"
  timeout -k 10 400 python benchmarks/rank_share/main.py --world 8 --steps 10 --warmup 3 --async-iters 3 \
      --restore-iters 2 --host-siblings 7 --sibling-dma-pass $dp > $O/rank_share_sib7_dma$dp.json \
      2> $O/rank_share_sib7_dma$dp.err || { echo RANKSHARE_FAIL; tail -20 $O/rank_share_sib7_dma$dp.err; exit 1; }
  tail -1 $O/rank_share_sib7_dma$dp.json
done
rm -rf bench_tmp
