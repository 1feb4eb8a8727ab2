#!/usr/bin/env python3
"""Where a rewrite take's time goes with and without the file mappings
(csrc/hsfmap.cpp): 5 takes of an 8 GiB bf16 state into one path per mode,
wall time per take, mapping-cache counters and timeline span totals."""

import glob
import json
import os
import sys
import time
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from hipsnapshot import Snapshot, StateDict  # noqa: E402
from hipsnapshot.knobs import override_tuning  # noqa: E402
from hipsnapshot.ops import native  # noqa: E402
from hipsnapshot.utils.tracing import timeline  # noqa: E402

D = os.environ.get("HSBENCH_DIR", "/tmp")
OUT = os.environ.get("PROBE_OUT", "gpurun_out/r5/k")
GiB = 1 << 30
NT = int(os.environ.get("PROBE_TENSORS", "64"))
comp = os.environ.get("PROBE_COMP", "none")
sd = StateDict({f"w{i}": torch.randn(8 * GiB // NT // 2, device="cuda").bfloat16()
                for i in range(NT)})
torch.cuda.synchronize()


def spans(prefix):
    tot = defaultdict(float)
    for f in glob.glob(prefix + "*.json"):
        with open(f) as fh:
            for e in json.load(fh)["traceEvents"]:
                tot[e["name"]] += e["dur"] / 1e3
        os.remove(f)
    keep = ("fmap", "fmap_commit", "dma", "write", "stage", "d2h", "hash_wait")
    return {k: round(v, 1) for k, v in tot.items() if k in keep}


for mode in os.environ.get("PROBE_MODES", "map,nomap").split(","):
    path = os.path.join(D, f"fm_{mode}")
    with override_tuning(file_map=(mode == "map")):
        for i in range(5):
            timeline.prefix = os.path.join(OUT, f"tl_{mode}_{i}")
            s0 = native.fmap_stats()
            t0 = time.perf_counter()
            Snapshot.take(path, {"sd": sd}, compression=comp)
            dt = time.perf_counter() - t0
            timeline.prefix = None
            s1 = native.fmap_stats()
            d = {k: s1[k] - s0[k] for k in ("hits", "maps", "drops", "misses")}
            print(json.dumps({"mode": mode, "take": i, "s": round(dt, 3),
                              "GBps": round(8 * GiB / dt / 1e9, 1), "fmap": d,
                              "mapped_GiB": round(s1["bytes"] / GiB, 2),
                              "span_ms_sum": spans(os.path.join(OUT, f"tl_{mode}_{i}"))}),
                  flush=True)
native.fmap_release(all_mappings=True)
