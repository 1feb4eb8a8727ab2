#!/bin/bash
# hsz_decode2 rate + LDS counters (one rocprofv3 --pmc pass, kernel trace only);
# COUNTERS overrides the counter list (<= 8 SQ_ counters), TAG the output dir
set -o pipefail
out=$PWD/gpurun_out/decode_pmc${TAG:-}
mkdir -p $out
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 120 python scripts/probes/hsz_decode_bench.py > $out/rate.json 2> $out/rate.err \
    || { echo RATE_FAIL; tail -20 $out/rate.err; exit 1; }
cat $out/rate.json
REPO=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --pmc ${COUNTERS:-SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_BUSY_CYCLES} \
    --kernel-include-regex "hsz_decode" --output-format csv -d $out/raw -o pmc \
    -- python3 $REPO/scripts/probes/hsz_decode_bench.py > $out/pmc.log 2>&1 || { echo PMC_FAIL; tail -20 $out/pmc.log; exit 1; }
cd $REPO
python3 - "$out" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
f = glob.glob(out + "/raw/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(float))
n = collections.Counter()
for r in csv.DictReader(open(f)):
    import re
    m = re.search(r"(hsz_decode2?g?)<(\d)>", r["Kernel_Name"])
    k = f"{m.group(1)}<{m.group(2)}>" if m else r["Kernel_Name"][:40]
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    if r["Counter_Name"] == "SQ_WAVES":
        n[k] += 1
with open(out + "/pmc_summary.txt", "w") as fo:
    for k, c in acc.items():
        line = f"{k}: dispatches={n[k]} " + " ".join(f"{a}={v / max(n[k], 1):.0f}" for a, v in sorted(c.items()))
        if c.get("SQ_INSTS_LDS"):
            line += f" conflict_cycles_per_lds_inst={c['SQ_LDS_BANK_CONFLICT'] / c['SQ_INSTS_LDS']:.2f}"
        print(line)
        fo.write(line + "\n")
PY
rm -rf $out/raw
