#!/bin/bash
# Session 2, call A: drain-helper GPU tests, full GPU suite, smoke, headline
# bench; the fp8 kernels (host-timed, rocprofv3 kernel stats, FETCH/WRITE
# counters) after the reciprocal-scale + packed-store change; UVM residency probe.
set -o pipefail
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD HIPSNAPSHOT_BENCH_DIR=$PWD/bench_tmp
REPO=$PWD
O=$PWD/gpurun_out/s2a
mkdir -p $O bench_tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -v -m gpu -k "drain_process or native_drain" \
    --timeout 120 --timeout-method thread > $O/pytest_helper.log 2>&1 \
    || { echo PYTEST_HELPER_FAIL; tail -40 $O/pytest_helper.log; exit 1; }
tail -2 $O/pytest_helper.log
TESTS=1 STEPS=10 bash scripts/gpu_check.sh || exit 1
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
timeout -k 10 180 python scripts/uvm_residency_probe.py > $O/uvm_probe.jsonl 2> $O/uvm_probe.err \
    || { echo UVM_PROBE_FAIL; tail -20 $O/uvm_probe.err; exit 1; }
cat $O/uvm_probe.jsonl
df -h /dev/shm /tmp $PWD | cat
free -g | cat
rm -rf bench_tmp
