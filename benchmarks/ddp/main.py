#!/usr/bin/env python3
"""Reference DDP benchmark config: 200 x 100 MB fp32 params (20 GB), replicated=["**"].

Reference: /root/reference/benchmarks/ddp/main.py:18-70 and README.md:9-24
(torchsnapshot 1 GPU 13.91 s, 8 GPUs 3.38 s on p4d; torch.save 32 s).
Reports save time / GB/s for hipsnapshot and for rank-0 torch.save.
"""

import argparse
import os
import shutil
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
from torch.nn.parallel import DistributedDataParallel as DDP  # noqa: E402

from common import Timer, emit, init_dist, log, max_over_ranks, sync  # noqa: E402
from hipsnapshot import Snapshot  # noqa: E402
from hipsnapshot.models.ddp_bench import ManyParams  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n-params", type=int, default=200)
    ap.add_argument("--param-mb", type=int, default=100)
    ap.add_argument("--work-dir", default=os.environ.get("HSBENCH_DIR", "/tmp"))
    ap.add_argument("--torch-save", action="store_true")
    ap.add_argument("--repeats", type=int, default=2)
    ap.add_argument("--compression", default="none", choices=["none", "hsz1"],
                    help="none = reference-format blobs (the published comparison)")
    ap.add_argument("--model", default="many_params", choices=["many_params", "llama3_8b"],
                    help="llama3_8b = BASELINE config 2 (Llama-3-8B DDP bf16, partitioned save)")
    args = ap.parse_args()
    rank, ws, dev = init_dist()
    if args.model == "llama3_8b":
        from hipsnapshot.models.llama import Llama, LlamaConfig, init_weights_

        with torch.device("meta"):
            inner = Llama(LlamaConfig.llama3_8b()).to(torch.bfloat16)
        inner.to_empty(device=dev)
        init_weights_(inner)
        nbytes = sum(p.numel() * p.element_size() for p in inner.parameters())
    else:
        inner = ManyParams(args.n_params, args.param_mb, dev)
        nbytes = args.n_params * args.param_mb * 1000 * 1000
    model = DDP(inner, device_ids=[dev.index] if dev.type == "cuda" else None,
                gradient_as_bucket_view=True)
    log(f"model size: {nbytes / 1e9:.1f} GB, world size {ws}")
    root = os.path.join(args.work_dir, "hs_ddp_bench")
    if rank == 0:
        shutil.rmtree(root, ignore_errors=True)
    sync(dev)
    best = None
    for i in range(args.repeats):
        sync(dev)
        with Timer() as t:
            Snapshot.take(os.path.join(root, "snap"), {"model": model}, replicated=["**"],
                          compression=args.compression)
            sync(dev)
        s = max_over_ranks(t.s, dev)
        log(f"hipsnapshot take {i}: {s:.2f}s ({nbytes / s / 1e9:.2f} GB/s)")
        best = s if best is None else min(best, s)
    ref = {1: 13.91, 8: 3.38}.get(ws) if args.model == "many_params" else None
    out = {"bench": "ddp_20gb_save" if args.model == "many_params" else "llama3_8b_ddp_save",
           "world_size": ws, "compression": args.compression, "bytes": nbytes,
           "seconds": round(best, 3),
           "GBps": round(nbytes / best / 1e9, 3),
           "reference_seconds": ref, "speedup_vs_reference": round(ref / best, 2) if ref else None}
    if args.torch_save and rank == 0:
        p = os.path.join(root, "torch_save.pt")
        with Timer() as t:
            torch.save(model.state_dict(), p)
        out["torch_save_seconds"] = round(t.s, 3)
    sync(dev)
    emit(out)
    if rank == 0:
        shutil.rmtree(root, ignore_errors=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
