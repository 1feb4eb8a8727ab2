#!/bin/bash
# Split-stream mode-2 encoder (hsz_encode2x, 4 threads per lane stream) vs the
# one-thread-per-stream encoder: codec GPU tests (bit-exact vs the reference
# encoder) with the split kernel, then the microbench kernel stats of both.
set -o pipefail
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD:$PYTHONPATH
CODEC_OUT=split_on bash scripts/gpu_codec.sh || exit 1
HIPSNAPSHOT_SPLIT_ENCODE=0 CODEC_OUT=split_off bash scripts/gpu_codec.sh || exit 1
