#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/blit
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD:$PYTHONPATH
for cfg in "X=0" "DEBUG_CLR_LIMIT_BLIT_WG=4" "DEBUG_CLR_LIMIT_BLIT_WG=16" "GPU_BLIT_ENGINE_TYPE=2" "GPU_BLIT_ENGINE_TYPE=1"; do
  env $cfg timeout -k 10 120 python scripts/d2h_probe.py >> gpurun_out/blit/probe.jsonl 2>> gpurun_out/blit/probe.err || { echo "FAIL $cfg"; tail -5 gpurun_out/blit/probe.err; exit 1; }
done
cat gpurun_out/blit/probe.jsonl
