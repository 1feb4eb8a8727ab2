"""Can GPU work written to a block through L2 reach HBM after the block was
freed and handed to another process as an uncached DMA target?  The
multi-process restore-pool trim failure (profiles/r5/trim/README.md) in its
simplest form: two writer processes fill plain blocks with a copy kernel
(through L2) and free them at once, while a reader process allocates
uncached blocks of the same size, uploads its own byte into them, sweeps L2
with unrelated kernels, reads them back and counts foreign bytes.  (The
in-process form -- free, reallocate uncached at the same VA, upload, read --
was clean: 20 of 20 rounds.)  Prints one JSON line."""

import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from hipsnapshot.ops import native  # noqa: E402



def _hip():
    torch.cuda.init()
    # the HIP runtime this process already runs (torch's), not another copy
    path = next(line.split()[-1] for line in open("/proc/self/maps") if "libamdhip64" in line)
    hip = ctypes.CDLL(path)
    hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
    hip.hipExtMallocWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t,
                                          ctypes.c_uint]
    hip.hipFree.argtypes = [ctypes.c_void_p]
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    return hip


N = 64 << 20


def writer(rounds: int, byte: int, q) -> None:
    """Kernel-fill plain blocks through L2 and free them at once."""
    torch.cuda.set_device(0)
    hip = _hip()
    native.require_gpu_lib()
    src = torch.full((N,), byte, dtype=torch.uint8, device="cuda")
    stream = torch.cuda.current_stream()
    for _ in range(rounds):
        x = ctypes.c_void_p()
        assert hip.hipMalloc(ctypes.byref(x), N) == 0
        b = native.CopyBatch()
        b.add_bytes(src.data_ptr(), x.value, N)
        keep = native.launch_packed(b.pack(), 0, int(stream.cuda_stream), sync=False)
        torch.cuda.synchronize()
        del keep
        assert hip.hipFree(x) == 0
    q.put({"writer_rounds": rounds})


def reader(rounds: int, byte: int, q) -> None:
    """Allocate uncached blocks, upload ``byte`` by DMA, read them back."""
    torch.cuda.set_device(0)
    hip = _hip()
    native.require_gpu_lib()
    host = torch.full((N,), byte, dtype=torch.uint8).pin_memory()
    out = torch.empty(N, dtype=torch.uint8)
    sweep = torch.empty(1 << 30, dtype=torch.uint8, device="cuda")
    res = {"rounds": 0, "bad_rounds": 0, "bad_bytes": 0}
    for _ in range(rounds):
        y = ctypes.c_void_p()
        assert hip.hipExtMallocWithFlags(ctypes.byref(y), N, 0x3) == 0
        assert hip.hipMemcpy(y, ctypes.c_void_p(host.data_ptr()), N, 1) == 0
        for _ in range(2):
            sweep.add_(1)
        torch.cuda.synchronize()
        assert hip.hipMemcpy(ctypes.c_void_p(out.data_ptr()), y, N, 2) == 0
        bad = int((out != byte).sum())
        res["rounds"] += 1
        res["bad_bytes"] += bad
        res["bad_rounds"] += int(bad > 0)
        assert hip.hipFree(y) == 0
    q.put(res)


if __name__ == "__main__":
    import multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=writer, args=(60, 0xA5, q)),
             ctx.Process(target=writer, args=(60, 0x5A, q)),
             ctx.Process(target=reader, args=(60, 0x3C, q))]
    for p in procs:
        p.start()
    got = [q.get(timeout=150) for _ in procs]
    for p in procs:
        p.join(30)
    print(json.dumps({"processes": got, "exitcodes": [p.exitcode for p in procs]}), flush=True)
