#!/bin/bash
# Native restore stage isolation: HIPSNAPSHOT_RESTORE_DEBUG 1 = no preads
# (uploads only), 2 = no uploads (reads only), at the W = 8 share and the
# full 1-GPU state (raw blobs: timing only, the bitwise check is meaningless
# there); then the hsz1 A/B with the process bound to the GPU's NUMA node.
set -o pipefail

out=gpurun_out/restore_probe
mkdir -p $out
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD:$PYTHONPATH HSBENCH_DIR=$PWD/bench_tmp
mkdir -p $HSBENCH_DIR
run() {  # name, env..., args...
  local name=$1; shift
  timeout -k 10 300 env "$@" > $out/$name.json 2> $out/$name.err || { echo FAIL $name; tail -20 $out/$name.err; return 1; }
  grep restore_ab $out/$name.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("'$name'", json.dumps(d["restore_ms"]), {k: {s: v.get(s) for s in ("wall", "upload_busy", "read", "slot_wait", "upload_wait", "first_upload")} for k, v in d.get("native_restore_stats", {}).items()})'
}
RS="python benchmarks/rank_share/main.py --steps 1 --warmup 1 --async-iters 1"
run w8_stage HIPSNAPSHOT_X=1 $RS --world 8 --compression none --restore-iters 4 --ab HIPSNAPSHOT_RESTORE_DEBUG=0,1,2 || exit 1
run w1_stage HIPSNAPSHOT_X=1 $RS --world 1 --compression none --restore-iters 3 --ab HIPSNAPSHOT_RESTORE_DEBUG=0,1,2 || exit 1
run w8_slot HIPSNAPSHOT_X=1 $RS --world 8 --compression hsz1 --restore-iters 4 --ab HIPSNAPSHOT_RESTORE_SLOT_BYTES=33554432,134217728 || exit 1
run w1_slot HIPSNAPSHOT_X=1 $RS --world 1 --compression hsz1 --restore-iters 3 --ab HIPSNAPSHOT_RESTORE_SLOT_BYTES=33554432,134217728 || exit 1
run w8_numa HIPSNAPSHOT_NUMA_BIND=1 $RS --world 8 --compression hsz1 --restore-iters 5 --ab HIPSNAPSHOT_NATIVE_RESTORE=1,0 || exit 1
run w1_numa HIPSNAPSHOT_NUMA_BIND=1 $RS --world 1 --compression hsz1 --restore-iters 3 --ab HIPSNAPSHOT_NATIVE_RESTORE=1,0 || exit 1
