"""Per-take fixed (byte-independent) overhead on the CPU: an FSDP2 Llama with
the Llama-3-8B layer structure (291 parameters, 32 blocks) but tiny widths,
so the planning / collective / commit path dominates.  Prints the mean take
time and the top cProfile entries.

    python scripts/profile_take_overhead.py [--takes 20] [--profile]
"""

from __future__ import annotations

import argparse
import cProfile
import os
import pstats
import shutil
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--takes", type=int, default=20)
    ap.add_argument("--profile", action="store_true")
    ap.add_argument("--compression", default="none")
    ap.add_argument("--optim", action="store_true", help="include AdamW state (3x the leaves)")
    ap.add_argument("--restore", action="store_true", help="time Snapshot.restore instead")
    args = ap.parse_args()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    import torch
    import torch.distributed as dist
    from torch.distributed.device_mesh import init_device_mesh

    from hipsnapshot import Snapshot
    from hipsnapshot.models.llama import LlamaConfig, build_fsdp_llama

    dist.init_process_group("gloo", rank=0, world_size=1)
    cfg = LlamaConfig(vocab_size=1024, dim=64, n_layers=32, n_heads=4, n_kv_heads=2,
                      ffn_dim=128, max_seq_len=64)
    model = build_fsdp_llama(cfg, torch.device("cpu"), torch.float32,
                             mesh=init_device_mesh("cpu", (1,)))
    print("params:", len(list(model.parameters())))
    root = tempfile.mkdtemp()
    app = {"model": model}
    if args.optim:
        opt = torch.optim.AdamW(model.parameters(), lr=1e-4)
        model(torch.randint(0, cfg.vocab_size, (1, 8))).sum().backward()
        opt.step()
        app["optim"] = opt
    Snapshot.take(os.path.join(root, "warm"), app, compression=args.compression)
    prof = cProfile.Profile() if args.profile else None
    times = []
    snap = Snapshot(os.path.join(root, "warm"))
    for i in range(args.takes):
        if prof:
            prof.enable()
        t0 = time.perf_counter()
        if args.restore:
            snap.restore(app)
        else:
            Snapshot.take(os.path.join(root, "s"), app, compression=args.compression)
        times.append(time.perf_counter() - t0)
        if prof:
            prof.disable()
    times.sort()
    print(f"mean {'restore' if args.restore else 'take'}: {sum(times) / len(times) * 1e3:.2f} ms, median "
          f"{times[len(times) // 2] * 1e3:.2f} ms, min {times[0] * 1e3:.2f} ms")
    if prof:
        pstats.Stats(prof).sort_stats("cumulative").print_stats(35)
    shutil.rmtree(root, ignore_errors=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
