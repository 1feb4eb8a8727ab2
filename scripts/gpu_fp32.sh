#!/bin/bash
# HSZ1 mode 2 for 4-byte elements: codec tests, microbench (+ kernel stats),
# fp32-master training overlap, then the full GPU suite / smoke / bench.
set -o pipefail
mkdir -p gpurun_out/overlap gpurun_out/fp32
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD:$PYTHONPATH HIPSNAPSHOT_BENCH_DIR=$PWD/bench_tmp
mkdir -p $HIPSNAPSHOT_BENCH_DIR
df -h $HIPSNAPSHOT_BENCH_DIR | tail -1
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -v -m gpu -k "hsz or compressed" \
    --timeout 120 --timeout-method thread > gpurun_out/fp32/pytest_hsz.log 2>&1 \
    || { echo PYTEST_FAIL; tail -40 gpurun_out/fp32/pytest_hsz.log; exit 1; }
tail -1 gpurun_out/fp32/pytest_hsz.log
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fp32/prof_micro -o micro \
    -- python3 benchmarks/microbench.py --skip-fs > gpurun_out/fp32/micro.jsonl 2> gpurun_out/fp32/micro.err \
    || { echo MICRO_FAIL; tail -30 gpurun_out/fp32/micro.err; exit 1; }
grep hsz gpurun_out/fp32/micro.jsonl
for c in hsz1 none; do
timeout -k 10 600 python benchmarks/train_overlap/main.py --layers 16 --seq 2048 --master-dtype fp32 \
    --compression $c > gpurun_out/overlap/fs_8b16L_fp32_$c.json 2> gpurun_out/overlap/fs_8b16L_fp32_$c.err \
    || { echo OVERLAP_FAIL; grep -v "^frame" gpurun_out/overlap/fs_8b16L_fp32_$c.err | tail -30; exit 1; }
tail -1 gpurun_out/overlap/fs_8b16L_fp32_$c.json
done
TESTS=1 STEPS=5 bash scripts/gpu_check.sh || exit 1
