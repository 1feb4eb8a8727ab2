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
        rows = list(csv.DictReader(f))
    # the trainer's stream / thread: the ones its per-step randint ran on
    mark = [r for r in rows if "random_from_to" in r["Kernel_Name"] or "randint" in r["Kernel_Name"]]
    if not mark:
        sys.exit("no per-step randint kernel found")
    t_stream = max({r["Stream_Id"] for r in mark}, key=lambda x: sum(r["Stream_Id"] == x for r in mark))
    t_thread = mark[-1]["Thread_Id"]
    other = defaultdict(lambda: [0, 0])
    for row in rows:
        name = row["Kernel_Name"]
        s, e = int(row["Start_Timestamp"]), int(row["End_Timestamp"])
        if ours(name) or row["Stream_Id"] != t_stream:
            if "hash64" in name:
                drain.append((s, e))
            k = name.split("(")[0][:80]
            other[k][0] += 1
            other[k][1] += e - s
            continue
        trainer.append((s, e, name))
        if row in mark:
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
    res["off_trainer_stream_kernels_ms"] = {k: {"n": v[0], "ms": round(v[1] / 1e6, 2)}
                                            for k, v in sorted(other.items(),
                                                               key=lambda x: -x[1][1])[:10]}
    api_path = path.replace("kernel_trace.csv", "hip_api_trace.csv")
    api = []
    if api_path != path:
        try:
            with open(api_path, newline="") as f:
                api = [r for r in csv.DictReader(f) if r.get("Thread_Id") == t_thread]
        except OSError:
            pass
    fcol = next((k for k in (api[0] if api else {}) if k in ("Function", "Operation")), None)
    if api:
        # the trainer thread's HIP calls per step: time inside the runtime
        # vs time between calls (Python, GIL, CPU share)
        api.sort(key=lambda r: int(r["Start_Timestamp"]))
        per = []
        j = 0
        for a, b in zip(markers, markers[1:]):
            while j < len(api) and int(api[j]["Start_Timestamp"]) < a:
                j += 1
            k, inside, n, fn = j, 0, 0, defaultdict(lambda: [0, 0])
            while k < len(api) and int(api[k]["Start_Timestamp"]) < b:
                d_ = int(api[k]["End_Timestamp"]) - int(api[k]["Start_Timestamp"])
                inside += d_
                n += 1
                f_ = fn[api[k][fcol] if fcol else "?"]
                f_[0] += 1
                f_[1] += d_
                k += 1
            during = any(s < b and e > a for s, e in windows)
            per.append((during, inside, n, fn))
        def agg(sel):
            if not sel:
                return None
            fns = defaultdict(lambda: [0, 0])
            for _, _, _, fn in sel:
                for name, (c, t) in fn.items():
                    fns[name][0] += c
                    fns[name][1] += t
            return {"in_runtime_ms": round(statistics.median(x[1] for x in sel) / 1e6, 3),
                    "calls": int(statistics.median(x[2] for x in sel)),
                    "top": {name: {"calls_per_step": round(c / len(sel), 1),
                                   "us_per_call": round(t / c / 1e3, 2)}
                            for name, (c, t) in sorted(fns.items(), key=lambda x: -x[1][1])[:6]}}
        res["trainer_thread_hip_api"] = {"baseline": agg([x for x in per[2:] if not x[0]]),
                                         "during_drain": agg([x for x in per if x[0]])}
    print(json.dumps(res, indent=1))
    if out_json:
        with open(out_json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
