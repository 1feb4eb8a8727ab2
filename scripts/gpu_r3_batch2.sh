#!/bin/bash
# Round 3 batch 2: mesh backend probe; fp8 kernel numerics + speed (host
# timed, rocprofv3 stats, FETCH/WRITE_SIZE passes); rank share at W=8 solo
# and with 7 host siblings; Llama-3-8B async_take + restore over S3.
set -o pipefail
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD HIPSNAPSHOT_BENCH_DIR=$PWD/bench_tmp
REPO=$PWD
O=$REPO/gpurun_out/r3b
mkdir -p $O/fp8 bench_tmp
echo "== mesh probe"
timeout -k 10 150 python scripts/mesh_backend_probe.py > $O/mesh_probe.log 2>&1; echo "mesh probe rc=$?"
grep -E "full ok|nccl|gloo" $O/mesh_probe.log | sort | uniq | head -20
echo "== (mx8 / fp8 tests ran in the full suite)"
echo "== fp8 kernels host-timed"
timeout -k 10 120 python scripts/fp8_kernels_bench.py > $O/fp8/host_timed.jsonl 2>&1 || { echo BENCH_FAIL; tail $O/fp8/host_timed.jsonl; exit 1; }
cat $O/fp8/host_timed.jsonl
cd /tmp && export TMPDIR=/tmp
echo "== rocprof kernel trace"
timeout -k 10 180 rocprofv3 --kernel-trace --stats --kernel-include-regex "hs_" --output-format csv \
    -d $O/fp8/trace -o fp8 -- python3 $REPO/scripts/fp8_kernels_bench.py \
    > $O/fp8/trace.log 2>&1 || { echo TRACE_FAIL; tail -20 $O/fp8/trace.log; exit 1; }
for pass in FETCH_SIZE WRITE_SIZE; do
  echo "== pmc $pass"
  tag=$(echo $pass | tr 'A-Z' 'a-z')
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $pass --kernel-include-regex "hs_" \
      --output-format csv -d $O/fp8/pmc_$tag -o pmc -- python3 $REPO/scripts/fp8_kernels_bench.py \
      > $O/fp8/pmc_$tag.log 2>&1 || { echo PMC_FAIL $tag; tail -20 $O/fp8/pmc_$tag.log; exit 1; }
done
cd $REPO
echo "== rank share W=8 solo + 7 host siblings"
timeout -k 10 400 python benchmarks/rank_share/main.py --world 8 --steps 10 --warmup 3 --async-iters 3 \
    --restore-iters 2 --host-siblings 7 > $O/rank_share_w8_sib7.json 2> $O/rank_share_w8_sib7.err \
    || { echo RANKSHARE_FAIL; tail -20 $O/rank_share_w8_sib7.err; exit 1; }
tail -1 $O/rank_share_w8_sib7.json
echo "== S3 Llama-3-8B"
timeout -k 10 400 python benchmarks/async_s3/main.py --iters 2 > $O/s3_8b.json 2> $O/s3_8b.err \
    || { echo S3_FAIL; tail -20 $O/s3_8b.err; exit 1; }
grep -E "async_take|restore" $O/s3_8b.err; tail -1 $O/s3_8b.json
rm -rf bench_tmp
