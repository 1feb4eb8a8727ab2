"""Per-rank phase split of one take, for multi-GPU runs whose curve must be
explained without another run (``bench.py``, ``benchmarks/rank_share``).

One take runs under ``timeline.capture()`` and ``getrusage``; its events
give, per rank: the wall time, how long the device -> host copies kept the
link busy (union of the ``d2h`` spans), how long storage writes were in
flight and at what page-cache rate, the CPU seconds the process spent, and
the milliseconds of each metadata collective (coalesce, replicated-path and
partition gathers, manifest gather, commit barriers).  ``skew`` condenses the
ranks into one line: max / median per field and the phase that separates the
slowest rank from the median one.
"""

from __future__ import annotations

import os
import resource
import statistics
import time
from typing import Callable, Dict, List, Sequence

from .tracing import timeline

# metadata / collective phases of a take (snapshot.py span names)
META_PHASES = ("coalesce", "replicated_entries", "partition", "barrier", "gather_manifest",
               "commit_barrier", "committed_barrier", "write_metadata", "uncommit")
# ... of which these run on a helper thread beside the writes (their time
# includes waiting for the slowest rank, not the take's critical path)
META_BACKGROUND = ("gather_manifest",)


def _union_s(events: Sequence[dict]) -> float:
    iv = sorted((e["ts"], e["ts"] + e["dur"]) for e in events)
    total, cur_s, cur_e = 0.0, None, None
    for s, e in iv:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                total += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        total += cur_e - cur_s
    return total / 1e6


def cpu_set() -> Dict[str, object]:
    """This process's CPU affinity: count and compact ranges."""
    cpus = sorted(os.sched_getaffinity(0))
    ranges, start, prev = [], None, None
    for c in cpus:
        if start is None:
            start = prev = c
        elif c == prev + 1:
            prev = c
        else:
            ranges.append(f"{start}-{prev}" if prev != start else str(start))
            start = prev = c
    if start is not None:
        ranges.append(f"{start}-{prev}" if prev != start else str(start))
    return {"n": len(cpus), "cpus": ",".join(ranges)}


def summarize(events: List[dict], wall_s: float, cpu_s: float) -> Dict[str, object]:
    d2h = [e for e in events if e.get("cat") == "d2h"]
    writes = [e for e in events if e.get("name") == "write" and e.get("cat") == "io"]
    drains = [e for e in events if e.get("name") == "native_drain"]
    d2h_bytes = sum(int(e["args"].get("bytes", 0)) for e in d2h)
    w_bytes = sum(int(e["args"].get("bytes", 0)) for e in writes + drains)
    w_busy = _union_s(writes + drains)
    meta = {}
    for e in events:
        if e.get("name") in META_PHASES:
            meta[e["name"]] = meta.get(e["name"], 0.0) + e["dur"] / 1e3
    return {
        "take_ms": round(wall_s * 1e3, 2),
        "d2h_busy_s": round(_union_s(d2h), 4),
        "d2h_GBps": round(d2h_bytes / max(_union_s(d2h), 1e-9) / 1e9, 2) if d2h else None,
        "write_busy_s": round(w_busy, 4),
        "write_bytes": w_bytes,
        "page_cache_GBps": round(w_bytes / max(w_busy, 1e-9) / 1e9, 2) if w_bytes else None,
        "cpu_s": round(cpu_s, 4),
        "cpu_s_per_GB": round(cpu_s / (w_bytes / 1e9), 4) if w_bytes else None,
        "meta_ms": {k: round(v, 2) for k, v in sorted(meta.items())},
        "meta_total_ms": round(sum(meta.values()), 2),
        "meta_critical_ms": round(sum(v for k, v in meta.items() if k not in META_BACKGROUND),
                                  2),
    }


def measure(take: Callable[[], object]) -> Dict[str, object]:
    """Run ``take()`` once with the timeline captured; its phase split."""
    r0 = resource.getrusage(resource.RUSAGE_SELF)
    with timeline.capture() as events:
        t0 = time.perf_counter()
        take()
        wall = time.perf_counter() - t0
    r1 = resource.getrusage(resource.RUSAGE_SELF)
    cpu = (r1.ru_utime - r0.ru_utime) + (r1.ru_stime - r0.ru_stime)
    out = summarize(events, wall, cpu)
    out["cpu_set"] = cpu_set()
    return out


def skew(per_rank: List[Dict[str, object]]) -> Dict[str, object]:
    """One line over the ranks: max / median of each timing field, the
    slowest rank, and the phase where it lost the most against the median."""
    fields = ("take_ms", "d2h_busy_s", "write_busy_s", "cpu_s", "meta_total_ms",
              "meta_critical_ms")
    out: Dict[str, object] = {}
    for f in fields:
        vals = [float(r[f]) for r in per_rank if r.get(f) is not None]
        if vals:
            med = statistics.median(vals)
            out[f"{f}_max_over_median"] = round(max(vals) / med, 3) if med else None
    takes = [float(r["take_ms"]) for r in per_rank]
    slow = max(range(len(takes)), key=lambda i: takes[i])
    out["slowest_rank"] = slow
    gaps = {}
    for f, scale in (("d2h_busy_s", 1e3), ("write_busy_s", 1e3), ("meta_critical_ms", 1.0)):
        vals = [float(r[f]) for r in per_rank if r.get(f) is not None]
        if len(vals) == len(per_rank):
            gaps[f] = (float(per_rank[slow][f]) - statistics.median(vals)) * scale
    if gaps:
        out["slowest_rank_phase"] = max(gaps, key=gaps.get)
        out["slowest_rank_phase_excess_ms"] = round(max(gaps.values()), 2)
    return out
