#!/bin/bash
# 8-rank gloo rehearsal of the multi-rank bench path on one GPU (all phases bitwise).
# (the DDP 20 GB phase needs ~39 GB per rank: it does not fit 8 ranks on one GPU)
set -o pipefail
mkdir -p gpurun_out/r5/o
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python bench.py --gpus 8 --backend gloo --steps 2 --warmup 1 --ddp-steps 0 --ddp-llama-layers 4 > gpurun_out/r5/o/reh8.log 2>&1; rc=$?
grep -v "amdgpu.ids\|Gloo\|^\[W" gpurun_out/r5/o/reh8.log | grep -E "^(warmup|step|async|restore|raw|fresh|DDP|elastic)" | cut -c1-220
tail -1 gpurun_out/r5/o/reh8.log > gpurun_out/r5/o/reh8.json
python - <<'PY'
import json
d = json.load(open("gpurun_out/r5/o/reh8.json"))
print({k: v for k, v in d.items() if k.endswith("ok") or k in ("value", "cold_time_to_unblock_ms", "time_to_unblock_ms", "world_size")})
PY
exit $rc
