"""Does the restore planner's per-region hsg_is_managed (hipPointerGetAttributes)
stall behind a concurrent restore prewarm (hipHostMalloc / hipMalloc of the
job's pools)?  Times 293 queries alone, then beside a prewarm thread."""
import json
import sys
import threading
import time

sys.path.insert(0, ".")
import torch

from hipsnapshot.engine import native_restore
from hipsnapshot.ops import native

torch.cuda.set_device(0)
ts = [torch.empty(1 << 20, dtype=torch.bfloat16, device="cuda") for _ in range(293)]
ptrs = [t.untyped_storage().data_ptr() for t in ts]
native.require_gpu_lib()
out = {}


def q():
    t0 = time.perf_counter()
    for p in ptrs:
        native.is_managed_ptr(p)
    return (time.perf_counter() - t0) * 1e3


out["first_ms"] = q()
out["alone_ms"] = [round(q(), 3) for _ in range(3)]
slot, _f, _n = native_restore.sizing(None)
res = {}


def pw():
    t0 = time.perf_counter()
    res["rc"] = native.restore_prewarm(0, 2 << 30, 2 << 30, slot, 2,
                                       native_restore.table_bytes(slot))
    res["ms"] = (time.perf_counter() - t0) * 1e3


th = threading.Thread(target=pw)
th.start()
time.sleep(0.0005)
out["beside_prewarm_ms"] = round(q(), 3)
th.join()
out["prewarm"] = res
t0 = time.perf_counter()
for t in ts:
    t.is_cuda and t.device.index
out["torch_attr_ms"] = round((time.perf_counter() - t0) * 1e3, 3)
print(json.dumps(out), flush=True)
