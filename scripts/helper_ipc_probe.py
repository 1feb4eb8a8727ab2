#!/usr/bin/env python3
"""Does the drain helper map an arena exported by this process?  One mode
per process (argv[1]): ``plain`` (no process group), ``nccl`` (RCCL process
group + one all_reduce first, as bench.py), ``gloo``.  Prints one JSON line."""

import json
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main() -> None:
    mode = sys.argv[1]
    opts = set(sys.argv[2:])  # numa, takes
    os.environ.update(HIPSNAPSHOT_DRAIN_PROCESS="1", HIPSNAPSHOT_DRAIN_HELPER_DEBUG="1",
                      HIPSNAPSHOT_DRAIN_HELPER_TIMEOUT_S="40",
                      HIPSNAPSHOT_DRAIN_HELPER_MAP_TIMEOUT_S="20")
    if "numa" in opts:
        from hipsnapshot.utils.affinity import bind_to_gpu_numa

        print(bind_to_gpu_numa(0), file=sys.stderr)
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    if mode in ("nccl", "gloo"):
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(29500 + os.getpid() % 1000))
        os.environ.update(RANK="0", WORLD_SIZE="1")
        if mode == "nccl":
            dist.init_process_group("nccl", device_id=dev)
            t = torch.ones(1, device=dev)
        else:
            dist.init_process_group("gloo")
            t = torch.ones(1)
        dist.all_reduce(t)
    from hipsnapshot import Snapshot, StateDict
    from hipsnapshot.engine import native_drain

    gib = int(os.environ.get("PROBE_GIB", "1"))
    w = torch.randn(gib * (256 << 20), device=dev)
    import ctypes

    libc = ctypes.CDLL(None)
    dumpable = libc.prctl(3, 0, 0, 0, 0)  # PR_GET_DUMPABLE
    with tempfile.TemporaryDirectory(dir=os.environ.get("HIPSNAPSHOT_BENCH_DIR")) as d:
        if "takes" in opts:
            sd = {"sd": StateDict(w=w.bfloat16(), v=torch.randn(64 << 20, device=dev))}
            for _ in range(5):
                Snapshot.take(os.path.join(d, "sync"), sd, compression="hsz1")
        t0 = time.perf_counter()
        err = None
        try:
            Snapshot.async_take(os.path.join(d, "s"), {"sd": StateDict(w=w)}).wait()
        except Exception as e:  # noqa: BLE001
            err = str(e).splitlines()[-1][:200]
        print(json.dumps({"mode": mode, "opts": sorted(opts), "s": round(time.perf_counter() - t0, 2),
                          "error": err, "where": native_drain.last_stats.get("where"),
                          "dumpable": dumpable}), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
