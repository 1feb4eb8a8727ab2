#!/bin/bash
# Training-overlap benchmark with short steps (seq 512: many steps inside one
# drain, so the per-step slowdown is measured over 15-25 steps instead of 3-6):
# split bf16 encoder on / off (interleaved, 2 runs each), then raw blobs.
set -o pipefail
out=gpurun_out/overlap_short
mkdir -p $out
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD:$PYTHONPATH HIPSNAPSHOT_BENCH_DIR=$PWD/bench_tmp
mkdir -p $HIPSNAPSHOT_BENCH_DIR
run() {  # name env...
  local name=$1; shift
  env "$@" timeout -k 10 600 python benchmarks/train_overlap/main.py --seq ${SEQ:-512} \
      --baseline-steps 10 ${ARGS:-} > $out/$name.json 2> $out/$name.err \
      || { echo OVERLAP_FAIL $name; grep -v "^frame" $out/$name.err | tail -30; return 1; }
  echo "$name $(tail -1 $out/$name.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ["baseline_step_ms","async_drain_s","steps_during_drain","step_ms_during_drain_mean","slowdown_during_drain"]})')"
}
for r in 1 2; do
  run split1_r$r HIPSNAPSHOT_SPLIT_ENCODE=1 || exit 1
  run split0_r$r HIPSNAPSHOT_SPLIT_ENCODE=0 || exit 1
done
ARGS="--compression none" run raw_r1 HIPSNAPSHOT_SPLIT_ENCODE=1 || exit 1
