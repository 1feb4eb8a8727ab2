#!/usr/bin/env python3
"""FSDP Llama async_take to S3 (BASELINE config 5) against the in-process fake
S3 server: time-to-unblock while the "trainer" keeps running, and total time.

``--model llama3_70b`` needs 8 GPUs x 17.6 GB; on one GPU use ``llama3_8b``
or the ``--layers`` override to scale the 70B geometry down.
"""

import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from common import emit, init_dist, log, max_over_ranks, sync  # noqa: E402
from hipsnapshot import Snapshot  # noqa: E402
from hipsnapshot.models.llama import LlamaConfig, build_fsdp_llama  # noqa: E402
from hipsnapshot.storage.fake_servers import FakeS3Server  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3_8b", choices=["llama3_8b", "llama3_70b"])
    ap.add_argument("--layers", type=int, default=None)
    args = ap.parse_args()
    rank, ws, dev = init_dist()
    from torch.distributed.device_mesh import init_device_mesh

    cfg = getattr(LlamaConfig, args.model)()
    if args.layers:
        cfg.n_layers = args.layers
    mesh = init_device_mesh(dev.type, (ws,))
    model = build_fsdp_llama(cfg, dev, torch.bfloat16, mesh=mesh)
    nbytes = sum(p._local_tensor.numel() * 2 for p in model.parameters())
    srv = FakeS3Server() if rank == 0 else None
    url = [srv.url if srv else None]
    dist.broadcast_object_list(url, src=0)
    opts = {"aws_access_key_id": "AKIDFAKE", "aws_secret_access_key": "fake-secret",
            "endpoint_url": url[0], "multipart_threshold": 64 << 20, "part_size": 64 << 20}
    sync(dev)
    t0 = time.perf_counter()
    pending = Snapshot.async_take("s3://ckpt/llama", {"model": model}, storage_options=opts)
    unblock = time.perf_counter() - t0
    # keep the "trainer" busy while the snapshot drains
    x = torch.randn(4096, 4096, device=dev, dtype=torch.bfloat16)
    steps = 0
    while not pending.done():
        x = x @ x.T
        x = x / x.norm()
        steps += 1
        if dev.type == "cuda":
            torch.cuda.synchronize()
    pending.wait()
    total = time.perf_counter() - t0
    unblock = max_over_ranks(unblock, dev)
    total = max_over_ranks(total, dev)
    emit({"bench": "async_take_s3", "model": args.model, "layers": cfg.n_layers, "world_size": ws,
          "bytes_per_rank": nbytes, "unblock_ms": round(unblock * 1e3, 1),
          "total_s": round(total, 3), "trainer_steps_during_drain": steps})
    sync(dev)
    if srv:
        srv.stop()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
