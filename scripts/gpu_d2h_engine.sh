#!/bin/bash
# D2H copy engine vs compute interference under runtime settings, then a
# kernel trace of two of them (are the copies blit kernels on the CUs?).
set -o pipefail
mkdir -p gpurun_out/d2h
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD:$PYTHONPATH
OUT=gpurun_out/d2h
timeout -k 10 120 python scripts/d2h_interference.py >> $OUT/probe.jsonl 2>> $OUT/probe.err || { echo FAIL default; tail -5 $OUT/probe.err; exit 1; }
GPU_BLIT_ENGINE_TYPE=1 timeout -k 10 120 python scripts/d2h_interference.py >> $OUT/probe.jsonl 2>> $OUT/probe.err || { echo FAIL bet1; tail -5 $OUT/probe.err; exit 1; }
GPU_BLIT_ENGINE_TYPE=2 timeout -k 10 120 python scripts/d2h_interference.py >> $OUT/probe.jsonl 2>> $OUT/probe.err || { echo FAIL bet2; tail -5 $OUT/probe.err; exit 1; }
HSA_ENABLE_SDMA=0 timeout -k 10 120 python scripts/d2h_interference.py >> $OUT/probe.jsonl 2>> $OUT/probe.err || { echo FAIL nosdma; tail -5 $OUT/probe.err; exit 1; }
cat $OUT/probe.jsonl
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $OUT/prof_default -o p \
    -- python3 scripts/d2h_interference.py > $OUT/prof_default.log 2>&1 || { echo PROF_FAIL; tail -5 $OUT/prof_default.log; exit 1; }
GPU_BLIT_ENGINE_TYPE=2 timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $OUT/prof_bet2 -o p \
    -- python3 scripts/d2h_interference.py > $OUT/prof_bet2.log 2>&1 || { echo PROF_FAIL2; tail -5 $OUT/prof_bet2.log; exit 1; }
for d in prof_default prof_bet2; do echo "== $d"; cat $OUT/$d/p_*_stats.csv | grep -i "copyBuffer\|MEMORY_COPY" | cut -c1-160 || true; done
