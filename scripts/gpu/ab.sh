#!/bin/bash
# Interleaved A/B of one knobs.TUNING constant on any benchmark script:
#   KNOB=name VALS="True False" N=3 OUT=gpurun_out/ab -- script.py args...
# (scripts/probes/with_tuning.py sets the constant in-process).
set -o pipefail
O=${OUT:-gpurun_out/ab}
mkdir -p $O
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD:$PYTHONPATH HSBENCH_DIR=$PWD/bench_tmp
mkdir -p $HSBENCH_DIR
[ "$1" = "--" ] && shift
for i in $(seq 1 ${N:-3}); do
  for v in ${VALS:-True False}; do
    f=$O/${KNOB}_${v}_$i
    timeout -k 10 ${T:-300} python scripts/probes/with_tuning.py $KNOB=$v -- "$@" > $f.json 2> $f.err \
        || { echo "FAIL $KNOB=$v run $i"; tail -20 $f.err; exit 1; }
    echo "$KNOB=$v run $i: $(tail -1 $f.json | cut -c1-400)"
  done
done
