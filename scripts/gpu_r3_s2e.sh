#!/bin/bash
# Session 2, call E: fp8 + UVM GPU tests, fp8 kernel timings (pipelined
# Hadamard quantizer), DLRM UVM restore into HBM-placed tables, 100 GB DLRM
# (BASELINE config 4 at full size, one GPU) with tables in UVM host DRAM,
# written to /dev/shm.
set -o pipefail
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD HIPSNAPSHOT_BENCH_DIR=$PWD/bench_tmp
O=$PWD/gpurun_out/s2e
mkdir -p $O bench_tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -v -m gpu -k "fp8 or mx8 or uvm" \
    --timeout 120 --timeout-method thread > $O/pytest_sub.log 2>&1 \
    || { echo PYTEST_FAIL; tail -40 $O/pytest_sub.log; exit 1; }
tail -2 $O/pytest_sub.log
timeout -k 10 120 python scripts/fp8_kernels_bench.py > $O/fp8_host_timed.jsonl 2>&1 \
    || { echo FP8_BENCH_FAIL; tail $O/fp8_host_timed.jsonl; exit 1; }
grep kernel $O/fp8_host_timed.jsonl
for pl in device default; do
  extra=""; [ $pl != default ] && extra="--uvm-place $pl"
  timeout -k 10 300 python benchmarks/dlrm_uvm/main.py --total-gb 8 --uvm $extra > $O/dlrm_uvm_$pl.json 2> $O/dlrm_uvm_$pl.err \
      || { echo DLRM_FAIL $pl; tail -20 $O/dlrm_uvm_$pl.err; exit 1; }
  tail -1 $O/dlrm_uvm_$pl.json
done
timeout -k 10 900 python benchmarks/dlrm_uvm/main.py --total-gb 100 --uvm --single-path --work-dir /dev/shm \
    > $O/dlrm_uvm_100gb.json 2> $O/dlrm_uvm_100gb.err \
    || { echo DLRM100_FAIL; tail -20 $O/dlrm_uvm_100gb.err; rm -rf /dev/shm/hs_dlrm; exit 1; }
tail -1 $O/dlrm_uvm_100gb.json
rm -rf /dev/shm/hs_dlrm bench_tmp
