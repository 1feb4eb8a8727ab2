"""Where a process's FIRST native restore spends its extra time: a 10 GB
raw read_object twice (cold, then warm) with the native job's phase stats,
and the time of a first 2 GiB uncached allocation / 768 MiB of pinned slots
in a fresh process."""
import json
import os
import shutil
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from hipsnapshot import Snapshot, StateDict  # noqa: E402
from hipsnapshot.engine import native_restore  # noqa: E402
from hipsnapshot.ops import native  # noqa: E402

mode = sys.argv[1] if len(sys.argv) > 1 else "read"
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
if mode == "alloc":
    torch.empty(1, device=dev)
    for what, fn in (("uncached_2GiB", lambda: native.UncachedBlock(0, 2 << 30)),
                     ("pinned_6x128MiB", lambda: [native.PinnedBuffer(128 << 20) for _ in range(6)])):
        t0 = time.perf_counter()
        keep = fn()
        print(json.dumps({what: round((time.perf_counter() - t0) * 1e3, 2)}), flush=True)
    sys.exit(0)
t = torch.randn(50000, 50000, device=dev)
root = os.path.join(os.environ.get("HSBENCH_DIR", "/tmp"), "cold_read_probe")
shutil.rmtree(root, ignore_errors=True)
Snapshot.take(root, {"sd": StateDict(t=t)})
import cProfile  # noqa: E402
import pstats  # noqa: E402

for i in range(3):
    out = torch.empty_like(t)
    torch.cuda.synchronize()
    prof = cProfile.Profile() if i == 0 else None
    t0 = time.perf_counter()
    if prof:
        prof.enable()
    Snapshot(root).read_object("0/sd/t", obj_out=out)
    torch.cuda.synchronize()
    if prof:
        prof.disable()
        pstats.Stats(prof, stream=sys.stderr).sort_stats("cumulative").print_stats(30)
    s = time.perf_counter() - t0
    print(json.dumps({"read": i, "ms": round(s * 1e3, 1), "GBps": round(t.numel() * 4 / s / 1e9, 2),
                      "native": native_restore.last_stats}), flush=True)
shutil.rmtree(root, ignore_errors=True)
