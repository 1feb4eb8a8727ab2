#!/usr/bin/env python3
"""read_object of a large GPU tensor with / without a memory budget (+ peak RSS).

Reference: /root/reference/benchmarks/load_tensor/main.py:24-61 (50000^2 fp32
= 10 GB GPU tensor, 100 MiB budget).  Tiled reads keep host memory under the
budget; every tile goes pinned -> H2D by DMA.
"""

import argparse
import os
import shutil
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from hipsnapshot import Snapshot, StateDict  # noqa: E402
from hipsnapshot.utils.rss_profiler import measure_rss_deltas  # noqa: E402
import time  # noqa: E402
import json  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=50000)
    ap.add_argument("--budget-mb", type=int, default=100)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--work-dir", default=os.environ.get("HSBENCH_DIR", "/tmp"))
    args = ap.parse_args()
    dev = torch.device("cuda" if torch.cuda.is_available() else "cpu")
    t = torch.randn(args.n, args.n, device=dev)
    root = os.path.join(args.work_dir, "hs_load_tensor")
    shutil.rmtree(root, ignore_errors=True)
    Snapshot.take(root, {"sd": StateDict(t=t)})
    nbytes = t.numel() * 4
    results = {}
    # alternated, twice each: the first read of a process pays its plans and
    # pools, whichever mode goes first; "GBps" is the better of the two
    out = torch.empty_like(t)
    for rnd in range(args.rounds):
        for name, budget in (("no_budget", None), ("budget", args.budget_mb << 20)):
            out.zero_()
            deltas = []
            if dev.type == "cuda":
                torch.cuda.synchronize()
            t0 = time.perf_counter()
            with measure_rss_deltas(deltas):
                Snapshot(root).read_object("0/sd/t", obj_out=out, memory_budget_bytes=budget)
                if dev.type == "cuda":
                    torch.cuda.synchronize()
            s = time.perf_counter() - t0
            assert torch.equal(out, t)
            r = results.setdefault(name, {"GBps_each": [], "peak_rss_delta_MB": 0.0})
            r["GBps_each"].append(round(nbytes / s / 1e9, 2))
            r["peak_rss_delta_MB"] = max(r["peak_rss_delta_MB"], round(max(deltas) / 2 ** 20, 1))
    for r in results.values():
        r["GBps"] = max(r["GBps_each"])
        r["seconds"] = round(nbytes / r["GBps"] / 1e9, 3)
    print(json.dumps({"bench": "load_tensor", "bytes": nbytes, **results}))
    shutil.rmtree(root, ignore_errors=True)


if __name__ == "__main__":
    main()
