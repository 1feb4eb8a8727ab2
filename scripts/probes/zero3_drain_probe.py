#!/usr/bin/env python3
"""Same-box A/B of the ZeRO-3 OPT-shape async save (benchmarks/deepspeed_opt)
between two source trees: ``zero3_drain_probe.py <tree root> <label>``
imports hipsnapshot from <tree root>, freezes the 4-layer OPT shape's
ZeRO-3 state (39.8 GB in HBM) with ``async_take`` and waits for the drain,
``--repeats`` times into the same path.  Prints one JSON line per save with
the native drain's per-phase seconds (``native_drain.last_stats``)."""

import argparse
import json
import os
import shutil
import sys
import time

ap = argparse.ArgumentParser()
ap.add_argument("root")
ap.add_argument("label")
ap.add_argument("--repeats", type=int, default=2)
ap.add_argument("--layers", type=int, default=4)
ap.add_argument("--work-dir", default=os.environ.get("HSBENCH_DIR", "/tmp"))
args = ap.parse_args()
sys.path.insert(0, os.path.abspath(args.root))

import torch  # noqa: E402

import hipsnapshot  # noqa: E402
from hipsnapshot import Snapshot  # noqa: E402
from hipsnapshot.engine import native_drain  # noqa: E402
from hipsnapshot.models.zero3 import EmulatedZero3Optimizer, OPTShape  # noqa: E402

assert os.path.dirname(hipsnapshot.__file__).startswith(os.path.abspath(args.root)), \
    hipsnapshot.__file__
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
shape = OPTShape(num_hidden_layers=args.layers, hidden_size=7168, num_attention_heads=56)
opt = EmulatedZero3Optimizer(shape, 0, 1, dev)
torch.cuda.synchronize()
root = os.path.join(args.work_dir, f"zero3_probe_{args.label}")
shutil.rmtree(root, ignore_errors=True)
for i in range(args.repeats):
    t0 = time.perf_counter()
    pending = Snapshot.async_take(os.path.join(root, "s"), {"optimizer": opt})
    t1 = time.perf_counter()
    pending.wait()
    t2 = time.perf_counter()
    nbytes = opt.nbytes()
    print(json.dumps({"label": args.label, "i": i, "unblock_ms": round((t1 - t0) * 1e3, 2),
                      "save_s": round(t2 - t0, 3), "GBps": round(nbytes / (t2 - t0) / 1e9, 2),
                      "drain": dict(native_drain.last_stats),
                      "env": {k: v for k, v in os.environ.items()
                              if k.startswith("HIPSNAPSHOT_DRAIN")}}), flush=True)
shutil.rmtree(root, ignore_errors=True)
