#!/bin/bash
# Whole GPU suite + smoke + bench on HEAD, then the seq-2048 drain-writers
# check (3 = new default vs 8) and one more seq-512 pair.
set -o pipefail
bash scripts/gpu_check.sh || exit 1
KNOB=HIPSNAPSHOT_DRAIN_WRITERS VALS="3 8" N=1 SEQ=2048 bash scripts/gpu_overlap_ab.sh || exit 1
mkdir -p gpurun_out/ov2048 && mv gpurun_out/overlap_ab/* gpurun_out/ov2048/
KNOB=HIPSNAPSHOT_DRAIN_WRITERS VALS="3 8" N=1 SEQ=512 bash scripts/gpu_overlap_ab.sh
