#!/bin/bash
# W-rank share restore (default W=8) under rocprofv3 kernel + memory-copy +
# HIP runtime traces: where the PCIe H2D idles during a restore and which
# runtime calls block.  Raw CSVs are reduced on the box by
# scripts/restore_trace_summary.py.
set -o pipefail
out=gpurun_out/restore_trace
mkdir -p $out
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD:$PYTHONPATH HSBENCH_DIR=$PWD/bench_tmp
mkdir -p $HSBENCH_DIR
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
tr=/tmp/rtrace_$$
HIPSNAPSHOT_TIMELINE=$PWD/$out/tl timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace \
    --output-format csv -d $tr -o rs -- python3 benchmarks/rank_share/main.py --world ${W:-8} \
    --steps 2 --warmup 1 --async-iters 1 --restore-iters 3 > $out/rs.json 2> $out/rs.err \
    || { echo RS_FAIL; tail -30 $out/rs.err; exit 1; }
tail -1 $out/rs.json
ls -la $tr
timeout -k 10 300 python3 scripts/restore_trace_summary.py $tr \
    > $out/summary.txt 2>&1 || { echo SUM_FAIL; tail -20 $out/summary.txt; exit 1; }
cat $out/summary.txt
rm -rf $tr
