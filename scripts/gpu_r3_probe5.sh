#!/bin/bash
# Where the seq-2048 drain's time goes (native drain phase stats), with and
# without blob checksums.
set -o pipefail
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD HIPSNAPSHOT_BENCH_DIR=$PWD/bench_tmp
O=$PWD/gpurun_out/r3l
mkdir -p $O bench_tmp
timeout -k 10 200 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 150 --timeout-method thread \
    -k "native_drain" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for mode in sum nosum; do
  envs=""; [ $mode = nosum ] && envs="HIPSNAPSHOT_CHECKSUM=0"
  echo "== $mode"
  env $envs timeout -k 10 500 python benchmarks/train_overlap/main.py --seq 2048 --checkpoints 3 \
      --gap-steps 10 --window-steps 20 --compression hsz1 > $O/overlap_$mode.json 2> $O/overlap_$mode.err \
      || { echo OVERLAP_FAIL; tail -20 $O/overlap_$mode.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/overlap_$mode.json').read().strip().splitlines()[-1]);print({k:d[k] for k in ['baseline_step_ms','async_drain_s_each','slowdown_during_drain','train_time_lost_local_ms']}); [print(x) for x in d['native_drain_stats_each']]"
done
rm -rf bench_tmp
