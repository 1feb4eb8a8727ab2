#!/bin/bash
# Session 2, call F: the full GPU suite, smoke and headline bench with the
# drain helper process on by default, plus a rocprofv3 kernel/copy profile
# of the bench.
set -o pipefail
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD
TESTS=1 STEPS=10 PROF=1 bash scripts/gpu_check.sh || exit 1
