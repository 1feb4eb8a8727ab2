"""Per-restore fixed (byte-independent) overhead at world size W on the CPU:
W gloo ranks, an FSDP2 Llama with the Llama-3-8B layer structure (291
parameters) but tiny widths, so metadata parsing, manifest-for-rank,
read planning, the read pipeline's per-blob costs and load_state_dict
dominate.  Rank 0 prints the median restore time and, with --profile, the
top cProfile entries of one restore.

    python scripts/profile_restore_overhead.py [--world 8] [--restores 10] [--profile]
"""

from __future__ import annotations

import argparse
import os
import statistics
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def work(path: str, restores: int, profile: bool, compression: str) -> None:
    import cProfile
    import pstats

    import torch
    import torch.distributed as dist
    from torch.distributed.device_mesh import init_device_mesh

    from hipsnapshot import Snapshot
    from hipsnapshot.models.llama import LlamaConfig, build_fsdp_llama

    ws = dist.get_world_size()
    cfg = LlamaConfig(vocab_size=1024, dim=64, n_layers=32, n_heads=4, n_kv_heads=2,
                      ffn_dim=128, max_seq_len=64)
    model = build_fsdp_llama(cfg, torch.device("cpu"), torch.float32,
                             mesh=init_device_mesh("cpu", (ws,)))
    app = {"model": model}
    Snapshot.take(path, app, compression=compression)
    times = []
    prof = cProfile.Profile() if profile and dist.get_rank() == 0 else None
    for i in range(restores):
        dist.barrier()
        if prof is not None and i == restores - 1:
            prof.enable()
        t0 = time.perf_counter()
        Snapshot(path).restore(app)
        times.append(time.perf_counter() - t0)
        if prof is not None and i == restores - 1:
            prof.disable()
    if dist.get_rank() == 0:
        print(f"world {ws}: restore median {statistics.median(times) * 1e3:.2f} ms, "
              f"min {min(times) * 1e3:.2f} ms", flush=True)
        if prof is not None:
            pstats.Stats(prof).sort_stats("cumulative").print_stats(35)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--restores", type=int, default=10)
    ap.add_argument("--profile", action="store_true")
    ap.add_argument("--compression", default="none")
    args = ap.parse_args()
    from hipsnapshot.utils.test_utils import run_distributed

    with tempfile.TemporaryDirectory() as d:
        run_distributed(work, args.world, os.path.join(d, "ck"), args.restores, args.profile,
                        args.compression)


if __name__ == "__main__":
    main()
