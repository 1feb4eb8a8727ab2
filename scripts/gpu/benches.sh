#!/bin/bash
# Every single-GPU benchmark, then the regression guard
# (scripts/check_thresholds.py against scripts/bench_thresholds.json).
#   OUT=gpurun_out/benches ONLY="bench dlrm_uvm ..." REPEAT=1 T=420
set -o pipefail
R=${OUT:-gpurun_out/benches}
mkdir -p $R
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD:$PYTHONPATH HSBENCH_DIR=$PWD/bench_tmp
mkdir -p $HSBENCH_DIR
want() { [ -z "${ONLY:-}" ] || [[ " $ONLY " == *" $1 "* ]]; }
run() {
  local name=$1; shift
  want $name || return 0
  for i in $(seq 1 ${REPEAT:-1}); do
    local tag=$name; [ "${REPEAT:-1}" = "1" ] || tag=${name}_$i
    echo "== $tag"
    timeout -k 10 ${T:-420} "$@" > $R/$tag.json 2> $R/$tag.err || { echo "FAIL $tag"; tail -20 $R/$tag.err; exit 1; }
    tail -1 $R/$tag.json | cut -c1-700
  done
}
run bench python bench.py --steps 5 --warmup 2
run ddp_20gb python benchmarks/ddp/main.py --repeats 3
run fsdp python benchmarks/fsdp/main.py
run load_tensor python benchmarks/load_tensor/main.py
run dlrm_uvm python benchmarks/dlrm_uvm/main.py --total-gb 8 --uvm ${DLRM_ARGS:-}
run dlrm_hbm python benchmarks/dlrm_uvm/main.py --total-gb 8
run deepspeed_opt python benchmarks/deepspeed_opt/main.py --layers 4
run cold_restore python benchmarks/cold_restore/main.py
run resnet_ddp python benchmarks/resnet_ddp/main.py
run share70b python benchmarks/rank_share/main.py --model llama3_70b --world 8 --steps 3 --warmup 1 --async-iters 2 --restore-iters 3
rm -rf $HSBENCH_DIR
[ -n "${ONLY:-}" ] || python scripts/check_thresholds.py $R
