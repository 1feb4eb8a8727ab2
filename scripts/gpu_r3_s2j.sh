#!/bin/bash
# Session 2, call J: bench.py with the drain helper again, with the new
# runtime-init / mapping markers and, if the helper stalls, the kernel wait
# channel of each of its threads.
set -o pipefail
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD HIPSNAPSHOT_BENCH_DIR=$PWD/bench_tmp
O=$PWD/gpurun_out/s2j
mkdir -p $O bench_tmp
( sleep 45
  for p in $(pgrep -f _hsdrain_helper); do
    echo "== helper $p: $(cat /proc/$p/status | grep -E '^State')"
    for t in /proc/$p/task/*; do echo "  task $(basename $t) $(cat $t/comm) wchan=$(cat $t/wchan) $(grep State $t/status)"; done
  done > $O/helper_wchan.txt 2>&1 ) &
W=$!
HIPSNAPSHOT_DRAIN_PROCESS=1 HIPSNAPSHOT_DRAIN_HELPER_DEBUG=1 HIPSNAPSHOT_DRAIN_HELPER_TIMEOUT_S=60 \
  timeout -k 10 150 python bench.py --steps 2 --warmup 1 --raw-steps 0 --fresh-steps 0 \
  --ddp-steps 0 --restore-iters 1 > $O/bench.json 2> $O/bench.err
rc=$?
echo "bench rc=$rc"
wait $W
grep -v "^frame" $O/bench.err | grep -E "hsdrain|async|warmup|step|Error|error" | tail -30
cat $O/helper_wchan.txt
tail -1 $O/bench.json
rm -rf bench_tmp
