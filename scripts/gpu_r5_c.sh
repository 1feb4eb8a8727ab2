#!/bin/bash
# After the round-5 refactor (host-only engines, pruned knobs, decoder
# variants removed): full GPU suite, smoke, headline bench, then the ZeRO-3
# save with the boosted-writer change (cold + rewrite) and the bench.
set -o pipefail
TESTS=1 STEPS=5 bash scripts/gpu_check.sh || exit 1
R=gpurun_out/r5/c
mkdir -p $R
export PYTHONUNBUFFERED=1 HSBENCH_DIR=$PWD/bench_tmp
mkdir -p $HSBENCH_DIR
timeout -k 10 300 python scripts/probes/zero3_drain_probe.py . head_boostfix > $R/zero3_after.jsonl 2> $R/zero3_after.err || { echo FAIL; tail -20 $R/zero3_after.err; exit 1; }
cut -c1-300 $R/zero3_after.jsonl
timeout -k 10 420 python benchmarks/deepspeed_opt/main.py --layers 4 > $R/deepspeed_opt.json 2> $R/deepspeed_opt.err || { echo FAIL; tail -20 $R/deepspeed_opt.err; exit 1; }
tail -1 $R/deepspeed_opt.json
rm -rf $HSBENCH_DIR
# the first take of a process vs later ones
mkdir -p $R/tl
HIPSNAPSHOT_TIMELINE=$PWD/$R/tl/b timeout -k 10 300 python bench.py --steps 2 --warmup 1 --async-iters 1 \
    --raw-steps 0 --fresh-steps 0 --ddp-steps 0 --ddp-llama-steps 0 --restore-iters 1 --verify-iters 0 \
    > $R/bench_tl.json 2> $R/bench_tl.err || { echo FAIL; tail -20 $R/bench_tl.err; exit 1; }
grep -E "warmup|step" $R/bench_tl.err | head
ls $R/tl | head -20
