#!/usr/bin/env python3
"""Split a training step's slowdown during an async-take drain into launch
gaps and longer kernels, from a ``rocprofv3 --kernel-trace`` CSV of
``benchmarks/train_overlap``.

Steps are cut at the trainer's per-step ``torch.randint`` kernel (the first
kernel of every step).  For each step: wall = start of the next step's
randint - start of this one; busy = union of the trainer's kernel intervals;
gaps = wall - busy (the GPU idle between the trainer's kernels: host launch
path, GIL, runtime locks, CPU share); kernel_sum = summed trainer kernel time
(longer kernels = HBM / L2 / CU contention).  A step is "during" a drain when
it overlaps a window of the drain's hash kernels (``hs_hash64``; windows are
split at gaps > 100 ms).  Prints medians of both classes and the kernels
whose median duration grew most.

    python scripts/overlap_trace_summary.py TRACE_kernel_trace.csv [--json out.json]
"""

from __future__ import annotations

import csv
import json
import statistics
import sys
from collections import defaultdict


def ours(name: str) -> bool:
    return "::hs_" in name or "::hsz_" in name or name.startswith(("hs_", "hsz_"))


def union(iv):
    tot, cs, ce = 0, None, None
    for s, e in sorted(iv):
        if ce is None or s > ce:
            if ce is not None:
                tot += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    if ce is not None:
        tot += ce - cs
    return tot


def main() -> None:
    path = sys.argv[1]
    out_json = sys.argv[sys.argv.index("--json") + 1] if "--json" in sys.argv else None
    trainer, drain, markers = [], [], []
    with open(path, newline="") as f:
        for row in csv.DictReader(f):
            name = row["Kernel_Name"]
            s, e = int(row["Start_Timestamp"]), int(row["End_Timestamp"])
            if ours(name):
                if "hash64" in name:
                    drain.append((s, e))
                continue
            trainer.append((s, e, name))
            if "randint" in name or ("random_from_to" in name) or \
                    ("distribution_elementwise" in name and "unsigned" in name.split("<")[1][:40]
                     if "<" in name else False):
                markers.append(s)
    markers.sort()
    drain.sort()
    windows = []
    for s, e in drain:
        if windows and s - windows[-1][1] < 100_000_000:
            windows[-1][1] = max(windows[-1][1], e)
        else:
            windows.append([s, e])
    trainer.sort()
    steps = []
    j = 0
    for a, b in zip(markers, markers[1:]):
        while j < len(trainer) and trainer[j][0] < a:
            j += 1
        k = j
        iv, ks, names = [], 0, []
        while k < len(trainer) and trainer[k][0] < b:
            s, e, n = trainer[k]
            iv.append((s, min(e, b)))
            ks += e - s
            names.append((n, e - s))
            k += 1
        busy = union(iv)
        during = any(s < b and e > a for s, e in windows)
        steps.append({"wall": b - a, "busy": busy, "gaps": b - a - busy, "ksum": ks,
                      "n": len(iv), "during": during, "names": names})

    def summ(sel):
        if not sel:
            return None
        return {k: round(statistics.median(x[k] for x in sel) / 1e6, 3)
                for k in ("wall", "busy", "gaps", "ksum")} | \
            {"steps": len(sel), "kernels": int(statistics.median(x["n"] for x in sel))}

    base = [x for x in steps[2:] if not x["during"]]  # first steps: warm-up
    dur = [x for x in steps if x["during"]]
    res = {"trace": path, "steps": len(steps), "drain_windows": len(windows),
           "drain_window_ms": [round((e - s) / 1e6, 1) for s, e in windows],
           "baseline_ms": summ(base), "during_drain_ms": summ(dur)}
    if base and dur:
        b, d = res["baseline_ms"], res["during_drain_ms"]
        res["slowdown_ms"] = {k: round(d[k] - b[k], 3) for k in ("wall", "busy", "gaps", "ksum")}
        per_b, per_d = defaultdict(list), defaultdict(list)
        for x in base:
            for n, t in x["names"]:
                per_b[n].append(t)
        for x in dur:
            for n, t in x["names"]:
                per_d[n].append(t)
        nb, nd = len(base), len(dur)
        grow = []
        for n in per_d:
            if n in per_b:
                db = sum(per_b[n]) / nb
                dd = sum(per_d[n]) / nd
                grow.append((dd - db, n, db, dd))
        grow.sort(reverse=True)
        res["kernel_time_growth_per_step_ms"] = [
            {"kernel": n[:120], "base_ms": round(db / 1e6, 3), "during_ms": round(dd / 1e6, 3),
             "growth_ms": round(g / 1e6, 3)} for g, n, db, dd in grow[:12]]
    print(json.dumps(res, indent=1))
    if out_json:
        with open(out_json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
