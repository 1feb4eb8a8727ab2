#!/usr/bin/env python3
"""Reduce a rocprofv3 trace of ``benchmarks/rank_share`` restores (kernel +
memory-copy + HIP runtime CSVs, ``scripts/gpu_restore_trace.sh``) to what
limits a restore: H2D busy time and idle gaps, decode / scatter kernel time,
and the HIP runtime calls that blocked for more than a millisecond.

Restore windows are found in the trace itself: host-to-device copies of at
least 1 MiB, clustered at gaps of more than 50 ms; the last cluster is the
last restore.

    python scripts/restore_trace_summary.py TRACE_DIR
"""

from __future__ import annotations

import csv
import glob
import json
import os
import sys
from collections import defaultdict


def _rows(pattern: str):
    files = glob.glob(pattern, recursive=True)
    if not files:
        return []
    with open(files[0], newline="") as f:
        return list(csv.DictReader(f))


def _col(row, *names):
    for n in names:
        for k in row:
            if k.lower() == n.lower():
                return row[k]
    for n in names:
        for k in row:
            if n.lower() in k.lower():
                return row[k]
    return None


def union(iv):
    tot, cs, ce, gaps = 0, None, None, []
    for s, e in sorted(iv):
        if ce is None or s > ce:
            if ce is not None:
                tot += ce - cs
                gaps.append((ce, s))
            cs, ce = s, e
        else:
            ce = max(ce, e)
    if ce is not None:
        tot += ce - cs
    return tot, gaps


def main() -> None:
    d = sys.argv[1]
    copies = _rows(os.path.join(d, "**", "*memory_copy_trace.csv"))
    kernels = _rows(os.path.join(d, "**", "*kernel_trace.csv"))
    api = _rows(os.path.join(d, "**", "*hip_api_trace.csv"))
    hdr = {"memory_copy": list(copies[0].keys()) if copies else None,
           "hip_api": list(api[0].keys()) if api else None}
    h2d = []
    for r in copies:
        direction = (_col(r, "Direction", "Operation", "Kind") or "").upper()
        if "HOST_TO_DEVICE" not in direction and "H2D" not in direction:
            continue
        s, e = int(_col(r, "Start_Timestamp")), int(_col(r, "End_Timestamp"))
        nb = _col(r, "Size", "Bytes", "Copy_Bytes")
        h2d.append((s, e, int(nb) if nb not in (None, "") else -1))
    h2d.sort()
    # copies of >= 1 MiB (or, without a size column, of >= 20 us)
    big = [c for c in h2d if c[2] >= (1 << 20) or (c[2] < 0 and c[1] - c[0] >= 20_000)]
    clusters = []
    for c in big:
        if clusters and c[0] - clusters[-1][-1][1] < 50_000_000:
            clusters[-1].append(c)
        else:
            clusters.append([c])
    out = {"h2d_copies": len(h2d), "restore_windows": len(clusters), "columns": hdr}
    if not clusters:
        print(json.dumps(out, indent=1))
        return
    last = clusters[-1]
    w0 = last[0][0]
    w1 = max(e for _, e, _ in last)
    in_w = [c for c in h2d if c[0] >= w0 - 5_000_000 and c[1] <= w1 + 5_000_000]
    busy, gaps = union([(s, e) for s, e, _ in in_w])
    nbytes = sum(max(n, 0) for _, _, n in in_w)
    out["last_restore"] = {
        "h2d_window_ms": round((w1 - w0) / 1e6, 2),
        "h2d_busy_ms": round(busy / 1e6, 2),
        "h2d_bytes": nbytes,
        "h2d_GBps_over_busy": round(nbytes / busy, 2) if busy else None,
        "h2d_GBps_over_window": round(nbytes / (w1 - w0), 2) if w1 > w0 else None,
        "h2d_copies": len(in_w),
        "h2d_idle_gaps_over_0.3ms": [(round((a - w0) / 1e6, 2), round((b - a) / 1e6, 2))
                                     for a, b in gaps if b - a > 300_000],
        "copy_ms_each": sorted((round((e - s) / 1e6, 2) for s, e, n in in_w
                                if n >= (1 << 20) or e - s >= 20_000),
                               reverse=True)[:12],
    }
    kt = defaultdict(lambda: [0, 0])
    kiv = []
    for r in kernels:
        s, e = int(_col(r, "Start_Timestamp")), int(_col(r, "End_Timestamp"))
        if s < w0 - 5_000_000 or e > w1 + 5_000_000:
            continue
        name = _col(r, "Kernel_Name") or "?"
        short = name.split("(")[0].replace("void ", "").replace("(anonymous namespace)::", "")
        kt[short][0] += 1
        kt[short][1] += e - s
        kiv.append((s, e))
    kbusy, _ = union(kiv)
    out["last_restore"]["kernel_busy_ms"] = round(kbusy / 1e6, 2)
    out["last_restore"]["kernels"] = {k: {"n": v[0], "ms": round(v[1] / 1e6, 2)}
                                      for k, v in sorted(kt.items(), key=lambda x: -x[1][1])[:10]}
    slow = []
    per_fn = defaultdict(lambda: [0, 0])
    for r in api:
        s, e = int(_col(r, "Start_Timestamp")), int(_col(r, "End_Timestamp"))
        if s < w0 - 10_000_000 or e > w1 + 5_000_000:
            continue
        fn = _col(r, "Function", "Operation") or "?"
        per_fn[fn][0] += 1
        per_fn[fn][1] += e - s
        if e - s > 1_000_000:
            slow.append((round((s - w0) / 1e6, 2), round((e - s) / 1e6, 2), fn,
                         _col(r, "Thread_Id")))
    out["last_restore"]["hip_api_total_ms"] = {k: {"n": v[0], "ms": round(v[1] / 1e6, 2)}
                                               for k, v in sorted(per_fn.items(),
                                                                  key=lambda x: -x[1][1])[:12]}
    out["last_restore"]["hip_api_calls_over_1ms"] = sorted(slow)[:40]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
