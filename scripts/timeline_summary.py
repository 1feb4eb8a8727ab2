#!/usr/bin/env python3
"""Summarise a hipsnapshot timeline (HIPSNAPSHOT_TIMELINE) trace file.

usage: timeline_summary.py TRACE.json [...]

Prints the planning phases, then for each span kind (stage / d2h / write /
read / ...) the count, bytes, the union of busy time, the first start and last
end relative to the trace origin, and the effective GB/s over the busy union.
"""

import json
import sys
from collections import defaultdict


def union(intervals):
    tot, cur_s, cur_e = 0.0, None, None
    for s, e in sorted(intervals):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def main():
    for f in sys.argv[1:]:
        ev = json.load(open(f))["traceEvents"]
        # keep the window of this operation's top-level phases (a background
        # async drain may have recorded spans into the same buffer)
        top = [e for e in ev if e["cat"] == "phase" and e["name"] in
               ("coalesce", "load_stateful")]
        if top:
            lo = min(e["ts"] for e in top)
            ev = [e for e in ev if e["ts"] >= lo]
        t0 = min(e["ts"] for e in ev)
        print(f"== {f}")
        for e in ev:
            if e["cat"] == "phase":
                print(f"  {e['name']:<20} start {(e['ts'] - t0) / 1e3:9.2f} ms  "
                      f"dur {e['dur'] / 1e3:9.2f} ms  {e.get('args') or ''}")
        groups = defaultdict(list)
        for e in ev:
            if e["cat"] != "phase":
                groups[e["name"]].append(e)
        for name, es in sorted(groups.items()):
            iv = [(e["ts"] - t0, e["ts"] - t0 + e["dur"]) for e in es]
            b = sum(e.get("args", {}).get("bytes", 0) for e in es)
            busy = union(iv) / 1e6
            durs = sorted(e["dur"] / 1e3 for e in es)
            print(f"  [{name:<11}] n={len(es):4d} bytes={b / 1e9:7.3f} GB busy={busy * 1e3:8.2f} ms "
                  f"first={min(s for s, _ in iv) / 1e3:8.2f} last_end={max(x for _, x in iv) / 1e3:8.2f} ms "
                  f"GB/s(busy)={b / busy / 1e9 if busy else 0:7.2f} "
                  f"dur med/max={durs[len(durs) // 2]:.2f}/{durs[-1]:.2f} ms")


if __name__ == "__main__":
    main()
