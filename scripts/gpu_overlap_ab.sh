#!/bin/bash
# train_overlap A/B of one env knob, runs interleaved: KNOB=NAME VALS="1 0" N=3 SEQ=512
set -o pipefail
out=gpurun_out/overlap_ab
mkdir -p $out
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD:$PYTHONPATH HSBENCH_DIR=$PWD/bench_tmp
mkdir -p $HSBENCH_DIR
K=${KNOB:-HIPSNAPSHOT_DRAIN_AVOID_CALLER_CORE}
for i in $(seq 1 ${N:-3}); do
  for v in ${VALS:-1 0}; do
    env $K=$v timeout -k 10 300 python benchmarks/train_overlap/main.py --seq ${SEQ:-512} \
        --checkpoints ${CKPT:-3} --gap-steps 10 --window-steps 30 > $out/${K}_${v}_$i.json 2> $out/${K}_${v}_$i.err \
        || { echo FAIL $v $i; grep -v "^frame" $out/${K}_${v}_$i.err | tail -20; exit 1; }
    echo "$K=$v run $i: $(tail -1 $out/${K}_${v}_$i.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ("baseline_step_ms","async_unblock_ms","async_drain_s","slowdown_during_drain","train_time_lost_vs_sync_take","train_time_lost_local_vs_sync_take","restore_bitwise_ok")})')"
  done
done
