#!/bin/bash
# fp32 split-stream encoder (HIPSNAPSHOT_SPLIT_ENCODE=2) vs hsz_encode2<4>:
# codec GPU tests bit-exact with it, microbench kernel stats of both.
set -o pipefail
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD:$PYTHONPATH
HIPSNAPSHOT_SPLIT_ENCODE=2 CODEC_OUT=split2 bash scripts/gpu_codec.sh || exit 1
HIPSNAPSHOT_SPLIT_ENCODE=1 CODEC_OUT=split1 bash scripts/gpu_codec.sh || exit 1
