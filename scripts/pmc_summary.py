#!/usr/bin/env python3
"""Condense rocprofv3 --pmc CSV output into a per-kernel summary (markdown + csv).

usage: pmc_summary.py OUT_PREFIX DIR [DIR ...]

Each DIR holds ``*_counter_collection.csv`` (and optionally
``*_kernel_trace.csv``) from one counter pass.  Per kernel name we report the
dispatch count, median duration and the median per-dispatch value of every
counter seen in any pass.  The raw CSVs can then be deleted (they are large).
"""

import csv
import glob
import os
import statistics
import sys
from collections import defaultdict


def short(name: str) -> str:
    name = name.replace("(anonymous namespace)::", "").replace("void ", "")
    name = name.split("(")[0]
    return name if len(name) <= 60 else name[:57] + "..."


def main():
    out_prefix, dirs = sys.argv[1], sys.argv[2:]
    vals = defaultdict(lambda: defaultdict(dict))  # kernel -> counter -> {dispatch: value}
    durs = defaultdict(dict)
    meta = {}
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    k = short(row.get("Kernel_Name", "?"))
                    disp = (d, row.get("Dispatch_Id"))
                    c = row.get("Counter_Name")
                    v = float(row.get("Counter_Value") or 0)
                    vals[k][c][disp] = vals[k][c].get(disp, 0.0) + v
                    meta.setdefault(k, {kk: row.get(kk) for kk in
                                        ("Grid_Size", "Workgroup_Size", "LDS_Block_Size",
                                         "Scratch_Size", "VGPR_Count", "Accum_VGPR_Count",
                                         "SGPR_Count")})
        for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    k = short(row.get("Kernel_Name", "?"))
                    try:
                        dt = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e3
                    except (KeyError, ValueError):
                        continue
                    durs[k][(d, row.get("Dispatch_Id"))] = dt
    counters = sorted({c for k in vals for c in vals[k]})
    rows = []
    for k in sorted(vals):
        n = max(len(vals[k][c]) for c in vals[k])
        r = {"kernel": k, "dispatches": n,
             "median_us": round(statistics.median(durs[k].values()), 2) if durs.get(k) else ""}
        for c in counters:
            xs = list(vals[k].get(c, {}).values())
            r[c] = round(statistics.median(xs), 1) if xs else ""
        r.update(meta.get(k, {}))
        rows.append(r)
    fields = list(rows[0].keys()) if rows else ["kernel"]
    with open(out_prefix + ".csv", "w", newline="") as fh:
        w = csv.DictWriter(fh, fieldnames=fields)
        w.writeheader()
        w.writerows(rows)
    with open(out_prefix + ".md", "w") as fh:
        fh.write("| " + " | ".join(fields) + " |\n")
        fh.write("|" + "---|" * len(fields) + "\n")
        for r in rows:
            fh.write("| " + " | ".join(str(r.get(f, "")) for f in fields) + " |\n")
    # per-dispatch table (dispatch order = program order; lets a caller map
    # dispatches of one kernel to the microbench case that issued them)
    disp_ids = sorted({(dk[1], k) for k in vals for c in vals[k] for dk in vals[k][c]},
                      key=lambda x: int(x[0] or 0))
    with open(out_prefix + "_dispatches.csv", "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["dispatch", "kernel", "dur_us"] + counters)
        for did, k in disp_ids:
            row = [did, k]
            dur = [v for (dd, i), v in durs.get(k, {}).items() if i == did]
            row.append(round(dur[0], 2) if dur else "")
            for c in counters:
                xs = [v for (dd, i), v in vals[k].get(c, {}).items() if i == did]
                row.append(xs[0] if xs else "")
            w.writerow(row)
    print(open(out_prefix + ".md").read())


if __name__ == "__main__":
    main()
