#!/bin/bash
# Same-box A/B of the 8-rank gloo rehearsal's blocking take: HEAD vs f9770d1 (ab_r3/old).
set -o pipefail
mkdir -p gpurun_out/r5/p
export PYTHONUNBUFFERED=1
ARGS="--gpus 8 --backend gloo --steps 3 --warmup 1 --async-iters 0 --raw-steps 0 --fresh-steps 0 --ddp-steps 0 --ddp-llama-steps 0 --verify-iters 0 --elastic-iters 0 --restore-iters 1"
for i in 1 2; do
  for t in head old; do
    if [ $t = head ]; then d=.; else d=ab_r3/old; fi
    (cd $d && timeout -k 10 400 python bench.py $ARGS --path /tmp/ab_$t > $GRAFT_REPO_ROOT/gpurun_out/r5/p/$t$i.log 2>&1) || { echo "$t$i failed"; tail -5 gpurun_out/r5/p/$t$i.log; exit 1; }
    echo "$t$i $(grep -E '^step' gpurun_out/r5/p/$t$i.log | tr '\n' ' ')"
  done
done
