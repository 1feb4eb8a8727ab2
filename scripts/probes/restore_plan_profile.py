"""cProfile of a process's FIRST restore into HBM (the cold planning path:
manifest, prepare_read, batching, the native job's plan), on a state with
the Llama-3-8B leaf structure (291 tensors) at small widths so per-leaf
costs dominate.  Prints the restore time, the planning phases' share and the
top functions by own time."""
import cProfile
import io
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from hipsnapshot import Snapshot, StateDict  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
g = torch.Generator(device=dev).manual_seed(0)
leaves = {"tok": torch.randn(4096, 256, device=dev, generator=g).bfloat16()}
for i in range(32):
    for n, shape in (("q", (256, 256)), ("k", (64, 256)), ("v", (64, 256)), ("o", (256, 256)),
                     ("gate", (896, 256)), ("up", (896, 256)), ("down", (256, 896)),
                     ("ln1", (256,)), ("ln2", (256,))):
        leaves[f"l{i}.{n}"] = torch.randn(*shape, device=dev, generator=g).bfloat16()
leaves["norm"] = torch.randn(256, device=dev, generator=g).bfloat16()
leaves["out"] = torch.randn(4096, 256, device=dev, generator=g).bfloat16()
root = os.path.join(os.environ.get("HSBENCH_DIR", "/tmp"), "restore_plan_profile")
comp = os.environ.get("COMPRESSION", "hsz1")
Snapshot.take(root, {"m": StateDict(**leaves)}, compression=comp)
torch.cuda.synchronize()
dst = StateDict(**{k: torch.zeros_like(v) for k, v in leaves.items()})
pr = cProfile.Profile()
t0 = time.perf_counter()
pr.enable()
Snapshot(root).restore({"m": dst})
pr.disable()
torch.cuda.synchronize()
cold = time.perf_counter() - t0
t0 = time.perf_counter()
Snapshot(root).restore({"m": dst})
torch.cuda.synchronize()
warm = time.perf_counter() - t0
assert all(torch.equal(dst[k], v) for k, v in leaves.items())
print(f"leaves={len(leaves)} compression={comp} cold_ms={cold * 1e3:.1f} warm_ms={warm * 1e3:.1f}")
s = io.StringIO()
pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(30)
print(s.getvalue())
s = io.StringIO()
pstats.Stats(pr, stream=s).sort_stats("cumulative").print_stats(40)
print(s.getvalue())
