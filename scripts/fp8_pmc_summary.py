#!/usr/bin/env python3
"""Summarise a gpu_r3_s2*.sh fp8 profile directory: per kernel (full
demangled name), rocprofv3 median duration and FETCH_SIZE / WRITE_SIZE
(KB per dispatch), the HBM traffic rate those counters imply, and the rate
the kernel's required bytes imply (the benchmark's 1 GiB of bf16 in, the
fp8 payload + scales out).

usage: fp8_pmc_summary.py <dir with fp8_trace/, fp8_pmc_fetch_size/, fp8_pmc_write_size/>
"""

import csv
import glob
import json
import re
import statistics
import sys
from collections import defaultdict


def _rows(pattern):
    out = []
    for f in glob.glob(pattern, recursive=True):
        with open(f, newline="") as fh:
            out += list(csv.DictReader(fh))
    return out


def main(d: str) -> None:
    durs = defaultdict(list)
    for r in _rows(f"{d}/fp8_trace/**/*kernel_trace.csv"):
        durs[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    ctr = defaultdict(lambda: defaultdict(list))
    for tag in ("fetch_size", "write_size"):
        for r in _rows(f"{d}/fp8_pmc_{tag}/**/*counter_collection.csv"):
            ctr[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = []
    for k, us in sorted(durs.items(), key=lambda kv: -statistics.median(kv[1])):
        if not re.search(r"::hs_(fp8|mx8)_\w+", k):
            continue
        med = statistics.median(us)
        rec = {"kernel": k, "n": len(us), "us_median": round(med, 1), "us_min": round(min(us), 1)}
        c = ctr.get(k)
        if c and c.get("FETCH_SIZE") and c.get("WRITE_SIZE"):
            fkb = statistics.median(c["FETCH_SIZE"])
            wkb = statistics.median(c["WRITE_SIZE"])
            rec.update(FETCH_KB=round(fkb), WRITE_KB=round(wkb),
                       TBps_counted=round((fkb + wkb) * 1024 / (med * 1e-6) / 1e12, 3))
        out.append(rec)
    for r in out:
        print(json.dumps(r))


if __name__ == "__main__":
    main(sys.argv[1])
