#!/bin/bash
# Session 2, call C: fp8 / UVM / drain-helper GPU tests, the streaming block
# fp8 quantizer (host-timed + rocprofv3 stats + FETCH/WRITE counters), DLRM
# UVM tables never placed / placed in host DRAM / placed in HBM, bench.py.
set -o pipefail
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD HIPSNAPSHOT_BENCH_DIR=$PWD/bench_tmp
REPO=$PWD
O=$PWD/gpurun_out/s2c
mkdir -p $O bench_tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -v -m gpu -k "fp8 or mx8 or uvm or drain_process" \
    --timeout 120 --timeout-method thread > $O/pytest_sub.log 2>&1 \
    || { echo PYTEST_FAIL; tail -40 $O/pytest_sub.log; exit 1; }
tail -2 $O/pytest_sub.log
timeout -k 10 120 python scripts/fp8_kernels_bench.py > $O/fp8_host_timed.jsonl 2>&1 \
    || { echo FP8_BENCH_FAIL; tail $O/fp8_host_timed.jsonl; exit 1; }
grep kernel $O/fp8_host_timed.jsonl
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats --kernel-include-regex "hs_" --output-format csv \
    -d $O/fp8_trace -o fp8 -- python3 $REPO/scripts/fp8_kernels_bench.py \
    > $O/fp8_trace.log 2>&1 || { echo TRACE_FAIL; tail -20 $O/fp8_trace.log; exit 1; }
for pass in FETCH_SIZE WRITE_SIZE; do
  tag=$(echo $pass | tr 'A-Z' 'a-z')
  timeout -s KILL 120 rocprofv3 --kernel-trace --stats --pmc $pass --kernel-include-regex "hs_" \
      --output-format csv -d $O/fp8_pmc_$tag -o pmc -- python3 $REPO/scripts/fp8_kernels_bench.py mx_e8m0 none hadamard32 \
      > $O/fp8_pmc_$tag.log 2>&1 || { echo PMC_FAIL $tag; tail -20 $O/fp8_pmc_$tag.log; exit 1; }
done
cd $REPO
for pl in default host device; do
  extra=""; [ $pl != default ] && extra="--uvm-place $pl"
  timeout -k 10 300 python benchmarks/dlrm_uvm/main.py --total-gb 8 --uvm $extra > $O/dlrm_uvm_$pl.json 2> $O/dlrm_uvm_$pl.err \
      || { echo DLRM_FAIL $pl; tail -20 $O/dlrm_uvm_$pl.err; exit 1; }
  tail -1 $O/dlrm_uvm_$pl.json
done
timeout -k 10 300 python bench.py --steps 5 --warmup 2 > $O/bench.json 2> $O/bench.err \
    || { echo BENCH_FAIL; tail -30 $O/bench.err; exit 1; }
cat $O/bench.json; grep -E "async" $O/bench.err
df -h /dev/shm /tmp $PWD | cat
free -g | cat
rm -rf bench_tmp
