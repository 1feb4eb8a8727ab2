#!/bin/bash
# Session 2, call S: HEAD check -- full GPU suite, smoke, headline bench, and a
# rocprofv3 kernel/copy-stats profile of the bench.
set -o pipefail
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD
TESTS=1 STEPS=10 PROF=1 bash scripts/gpu_check.sh || exit 1
