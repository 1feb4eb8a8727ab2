"""Allocator state before the first async_take of the headline bench: why does
the first HBM freeze take >100 ms?  Prints reserved / allocated / device-free
memory after sync takes, then times the arena allocation alone."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29571")
import torch
import torch.distributed as dist
from torch.distributed.device_mesh import init_device_mesh

from hipsnapshot import Snapshot
from hipsnapshot.models.llama import LlamaConfig, build_fsdp_llama


def state(tag):
    torch.cuda.synchronize()
    free, total = torch.cuda.mem_get_info()
    st = torch.cuda.memory_stats()
    print(f"{tag}: reserved {torch.cuda.memory_reserved() / 1e9:.2f} GB, allocated "
          f"{torch.cuda.memory_allocated() / 1e9:.2f} GB, device free {free / 1e9:.1f} / "
          f"{total / 1e9:.1f} GB, segments {st.get('segment.all.current', 0)}, "
          f"largest inactive split {st.get('inactive_split_bytes.all.current', 0) / 1e9:.2f} GB, "
          f"num_alloc_retries {st.get('num_alloc_retries', 0)}", flush=True)


def timed_alloc(nbytes, tag):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    a = torch.empty(nbytes, dtype=torch.uint8, device="cuda:0")
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    print(f"{tag}: torch.empty({nbytes / 1e9:.1f} GB) {1e3 * (t1 - t0):.1f} ms "
          f"(+sync {1e3 * (time.perf_counter() - t1):.1f} ms)", flush=True)
    return a


dist.init_process_group("nccl", rank=0, world_size=1)
torch.cuda.set_device(0)
model = build_fsdp_llama(LlamaConfig.llama3_8b(), torch.device("cuda:0"), torch.bfloat16,
                         mesh=init_device_mesh("cuda", (1,)))
path = os.path.join(os.environ.get("HSBENCH_DIR", "/tmp"), "probe")
nbytes = 16060522496
state("after model")
a = timed_alloc(nbytes, "fresh process")
del a
torch.cuda.empty_cache()
for i in range(3):
    Snapshot.take(path, {"model": model}, compression=os.environ.get("COMP", "hsz1"))
    state(f"after sync take {i}")
a = timed_alloc(nbytes, "after sync takes")
del a
a = timed_alloc(nbytes, "again (cached)")
del a
torch.cuda.empty_cache()
state("after empty_cache")
a = timed_alloc(nbytes, "after empty_cache")
del a
dist.destroy_process_group()
