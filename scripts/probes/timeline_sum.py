#!/usr/bin/env python3
"""Sum the spans of timeline dumps (HIPSNAPSHOT_TIMELINE=<prefix>): per file,
total / count / max milliseconds of each span name, and the wall extent."""

import glob
import json
import sys
from collections import defaultdict

for f in sorted(glob.glob(sys.argv[1] + "*.json")):
    ev = json.load(open(f))["traceEvents"]
    tot, cnt, mx = defaultdict(float), defaultdict(int), defaultdict(float)
    for e in ev:
        d = e["dur"] / 1e3
        tot[e["name"]] += d
        cnt[e["name"]] += 1
        mx[e["name"]] = max(mx[e["name"]], d)
    wall = (max(e["ts"] + e["dur"] for e in ev) - min(e["ts"] for e in ev)) / 1e3
    top = sorted(tot, key=lambda k: -tot[k])[:12]
    print(f.split("/")[-1], f"wall {wall:.1f} ms",
          {k: (round(tot[k], 1), cnt[k], round(mx[k], 1)) for k in top})
