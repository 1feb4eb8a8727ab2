#!/bin/bash
# codec kernels only: bit-exact / round-trip tests, then the microbench with kernel stats
set -o pipefail
OUT=gpurun_out/${CODEC_OUT:-codec}
mkdir -p $OUT
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -v -m gpu -k "hsz or compressed" \
    --timeout 120 --timeout-method thread > $OUT/pytest_hsz.log 2>&1 \
    || { echo PYTEST_FAIL; grep -E "FAILED|Error|assert" $OUT/pytest_hsz.log | head -20; exit 1; }
tail -1 $OUT/pytest_hsz.log
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_micro -o micro \
    -- python3 benchmarks/microbench.py --skip-fs > $OUT/micro.jsonl 2> $OUT/micro.err \
    || { echo MICRO_FAIL; tail -30 $OUT/micro.err; exit 1; }
grep hsz $OUT/micro.jsonl
python3 - "$OUT/prof_micro/micro_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "hsz" in r["Name"]:
        print(r["Name"].split("::")[1][:24], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us")
PY
