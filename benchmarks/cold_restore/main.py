"""Restore in a FRESH process (the restart-after-failure case).

``bench.py`` times restores in the process that just saved: the pinned host
pool, the device caching allocator and the HIP code objects are all warm.
A job restarting from a checkpoint has none of that.  This benchmark saves
the Llama-3-8B FSDP state in one process, then restores it in a second,
fresh process (random-init with the same seed, so the restored shards are
checked bitwise against a regenerated copy) and times its first and second
restore.  The checkpoint files are still in the page cache (dropping it
needs root), so storage reads are warm in both cases.

    python benchmarks/cold_restore/main.py [--compression hsz1] [--dir DIR]
"""

from __future__ import annotations

import argparse
import json
import os
import shutil
import subprocess
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))


def _init(port: int):
    import torch
    import torch.distributed as dist

    os.environ.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", device_id=dev)
    from torch.distributed.device_mesh import init_device_mesh

    from hipsnapshot.models.llama import LlamaConfig, build_fsdp_llama

    torch.manual_seed(1234)
    mesh = init_device_mesh("cuda", (1,))
    model = build_fsdp_llama(LlamaConfig.llama3_8b(), dev, torch.bfloat16, mesh=mesh)
    torch.cuda.synchronize()
    return model


def _child(args) -> None:
    import torch
    import torch.distributed as dist

    from hipsnapshot import Snapshot
    from hipsnapshot.ops import native

    t_start = time.perf_counter()
    model = _init(args.port)
    native.require_gpu_lib()
    app_state = {"model": model}
    nbytes = sum(p._local_tensor.numel() * p._local_tensor.element_size()
                 for p in model.parameters())
    out = {"role": args.role, "model_build_s": round(time.perf_counter() - t_start, 2)}
    if args.role == "save":
        t = time.perf_counter()
        Snapshot.take(args.path, app_state, compression=args.compression)
        out["take_s"] = round(time.perf_counter() - t, 3)
    else:
        named = list(model.named_parameters())
        refs = [p._local_tensor.clone() for _, p in named]
        times = []
        ok = True
        prof_out = os.environ.get("HSBENCH_PROFILE")  # cProfile of each restore
        for i in range(args.restores):
            for _, p in named:
                p._local_tensor.zero_()
            torch.cuda.synchronize()
            prof = None
            if prof_out:
                import cProfile

                prof = cProfile.Profile()
                prof.enable()
            t = time.perf_counter()
            Snapshot(args.path).restore(app_state)
            torch.cuda.synchronize()
            times.append(time.perf_counter() - t)
            if prof is not None:
                import io
                import pstats

                prof.disable()
                buf = io.StringIO()
                st = pstats.Stats(prof, stream=buf)
                st.sort_stats("cumulative").print_stats(60)
                st.sort_stats("tottime").print_stats(40)
                with open(f"{prof_out}.restore{i}.txt", "w") as f:
                    f.write(buf.getvalue())
            named = list(model.named_parameters())
            ok = ok and all(torch.equal(r, p._local_tensor) for (_, p), r in zip(named, refs))
        out.update({"restore_s_each": [round(x, 4) for x in times],
                    "restore_GBps_each": [round(nbytes / x / 1e9, 2) for x in times],
                    "restore_bitwise_ok": ok, "checkpoint_bytes": nbytes})
    print(json.dumps(out), flush=True)
    dist.destroy_process_group()


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--role", default=None, choices=["save", "restore"])
    ap.add_argument("--path", default=None)
    ap.add_argument("--dir", default=os.environ.get("HSBENCH_DIR", "/tmp"))
    ap.add_argument("--compression", default="hsz1", choices=["none", "hsz1"])
    ap.add_argument("--restores", type=int, default=2)
    ap.add_argument("--port", type=int, default=29571)
    args = ap.parse_args()
    if args.role is not None:
        _child(args)
        return
    root = os.path.join(args.dir, "cold_restore")
    shutil.rmtree(root, ignore_errors=True)
    os.makedirs(root)
    path = os.path.join(root, "ckpt")
    results = []
    try:
        # each role in its own child process: the restore one starts cold
        for role, port in (("save", args.port), ("restore", args.port + 1)):
            cmd = [sys.executable, os.path.abspath(__file__), "--role", role, "--path", path,
                   "--compression", args.compression, "--restores", str(args.restores),
                   "--port", str(port)]
            r = subprocess.run(cmd, stdout=subprocess.PIPE, text=True, timeout=600)
            if r.returncode != 0:
                raise SystemExit(f"{role} child failed with exit code {r.returncode}")
            results.append(json.loads(r.stdout.strip().splitlines()[-1]))
    finally:
        shutil.rmtree(root, ignore_errors=True)
    print(json.dumps({"bench": "cold_restore", "model": "Llama-3-8B", "parallelism": "fsdp1",
                      "compression": args.compression, "save": results[0],
                      "restore": results[1]}), flush=True)


if __name__ == "__main__":
    main()
