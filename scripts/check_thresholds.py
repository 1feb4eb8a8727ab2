#!/usr/bin/env python3
"""Regression guard for the single-GPU benchmark set (scripts/gpu/benches.sh):
``check_thresholds.py <dir with one JSON per benchmark>`` compares each
metric with its floor (or ceiling) in scripts/bench_thresholds.json and exits 1
when any is missed.  Floors sit ~20 % under the round-5 measurements:
boxes differ by a few percent, a code regression by more."""

import json
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def last_json(path):
    with open(path) as f:
        lines = [ln for ln in f.read().splitlines() if ln.strip().startswith("{")]
    return json.loads(lines[-1])


def main() -> int:
    d = sys.argv[1]
    with open(os.path.join(HERE, "scripts", "bench_thresholds.json")) as f:
        spec = json.load(f)
    bad = 0
    for bench, metrics in spec.items():
        p = os.path.join(d, f"{bench}.json")
        if not os.path.exists(p):
            print(f"MISSING {bench}")
            bad += 1
            continue
        got = last_json(p)
        for key, rule in metrics.items():
            v = got.get(key)
            if isinstance(v, list):  # per-iteration values: the worst one counts
                v = (min(v) if "min" in rule else max(v)) if v else None
            ok = v is not None and (v >= rule["min"] if "min" in rule else v <= rule["max"])
            bad += not ok
            bound = f">= {rule['min']}" if "min" in rule else f"<= {rule['max']}"
            print(f"{'ok  ' if ok else 'FAIL'} {bench}.{key} = {v} ({bound})")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
