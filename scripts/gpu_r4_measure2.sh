#!/bin/bash
set -o pipefail
bash scripts/gpu_restore_trace.sh || exit 1
bash scripts/gpu_overlap_trace.sh
