#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r5/n
export PYTHONUNBUFFERED=1
HIPSNAPSHOT_TIMELINE=gpurun_out/r5/n/bt timeout -k 10 600 python bench.py > gpurun_out/r5/n/bench.log 2>&1 || { tail -20 gpurun_out/r5/n/bench.log; exit 1; }
grep -E "^(warmup|step|async|raw|fresh|DDP)" gpurun_out/r5/n/bench.log | cut -c1-200
ls gpurun_out/r5/n | head -50 > gpurun_out/r5/n/files.txt
python scripts/probes/timeline_sum.py gpurun_out/r5/n/bt.rank0.take > gpurun_out/r5/n/take_sums.txt 2>&1
awk '{print $1, $2, $3, $4}' gpurun_out/r5/n/take_sums.txt
rm -f gpurun_out/r5/n/bt.*.json
