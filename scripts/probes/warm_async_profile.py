#!/usr/bin/env python3
"""Where a WARM async_take (plan cached, arena kept) spends its unblock time:
FSDP Llama-3-8B on one GPU, 5 untimed async takes, then 20 timed ones; the
last 10 under cProfile (--profile).  Prints the unblock times and the top
entries by cumulative and own time (of the async_take calls only)."""

import cProfile
import io
import os
import pstats
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29534")
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
torch.cuda.set_device(0)
from hipsnapshot.utils.affinity import bind_to_gpu_numa  # noqa: E402

bind_to_gpu_numa(0)
from torch.distributed.device_mesh import init_device_mesh  # noqa: E402

from hipsnapshot import Snapshot  # noqa: E402
from hipsnapshot.models.llama import LlamaConfig, build_fsdp_llama  # noqa: E402

model = build_fsdp_llama(LlamaConfig.llama3_8b(), torch.device("cuda", 0), torch.bfloat16,
                         mesh=init_device_mesh("cuda", (1,)))
torch.cuda.synchronize()
D = os.environ.get("HSBENCH_DIR", "/tmp")
app = {"model": model}
Snapshot.take(os.path.join(D, "w"), app, compression="hsz1")
for _ in range(5):
    Snapshot.async_take(os.path.join(D, "wa"), app, compression="hsz1").wait()
prof = cProfile.Profile() if "--profile" in sys.argv else None
times = []
for i in range(20):
    torch.cuda.synchronize()
    if prof and i >= 10:
        prof.enable()
    t0 = time.perf_counter()
    pending = Snapshot.async_take(os.path.join(D, "wa"), app, compression="hsz1")
    times.append((time.perf_counter() - t0) * 1e3)
    if prof and i >= 10:
        prof.disable()
    pending.wait()
print({"warm_unblock_ms_median": round(statistics.median(times), 3),
       "each": [round(t, 2) for t in times], "profiled": prof is not None}, flush=True)
if prof:
    for key in ("cumulative", "tottime"):
        s = io.StringIO()
        pstats.Stats(prof, stream=s).sort_stats(key).print_stats(35)
        print(s.getvalue())
