#!/usr/bin/env python3
"""Where the FIRST async_take of a process spends its unblock time: the bench's
sequence (FSDP Llama-3-8B on one GPU, one blocking take first), then the cold
async_take under cProfile (--profile) or timed plainly; a second, warm
async_take for comparison."""

import cProfile
import io
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29533")
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
if "--async-first" not in sys.argv:  # (the bench's order: a blocking take first)
    Snapshot.take(os.path.join(D, "c"), {"model": model}, compression="hsz1")
torch.cuda.synchronize()
prof = "--profile" in sys.argv
if os.environ.get("PROBE_TL"):
    from hipsnapshot.utils.tracing import timeline

    timeline.prefix = os.environ["PROBE_TL"]
p = cProfile.Profile() if prof else None
t0 = time.perf_counter()
if p:
    p.enable()
pending = Snapshot.async_take(os.path.join(D, "ca"), {"model": model}, compression="hsz1")
if p:
    p.disable()
cold = (time.perf_counter() - t0) * 1e3
pending.wait()
t0 = time.perf_counter()
pending = Snapshot.async_take(os.path.join(D, "ca"), {"model": model}, compression="hsz1")
warm = (time.perf_counter() - t0) * 1e3
pending.wait()
print({"cold_unblock_ms": round(cold, 2), "warm_unblock_ms": round(warm, 2), "profiled": prof},
      flush=True)
if p:
    for key in ("cumulative", "tottime"):
        s = io.StringIO()
        pstats.Stats(p, stream=s).sort_stats(key).print_stats(45)
        print(s.getvalue(), flush=True)
dist.destroy_process_group()
