#!/usr/bin/env python3
"""FSDP Llama ``async_take`` to S3 and restore from it (BASELINE config 5).

The S3 endpoint is the SigV4-verifying fake server running in ITS OWN
PROCESS (``FakeS3Process``), so the numbers measure the client: the blocking
keep-alive connection pool of ``storage/s3.py`` -- parallel multipart PUTs
sent straight from the pinned staging buffers, parallel ranged GETs received
straight into the pinned read buffers.  Loopback TCP, no TLS, no network.

Reports time-to-unblock, the background drain's write GB/s (logical model
bytes / async_take-to-commit time), and restore GB/s with a bitwise check.
Reference path: `/root/reference/torchsnapshot/storage_plugins/s3.py:39-66`.

``--model llama3_70b`` needs 8 GPUs x 17.6 GB; on one GPU use ``llama3_8b``
or ``--layers`` to scale the geometry down.
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
from hipsnapshot.storage.fake_servers import FakeS3Process  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3_8b", choices=["llama3_8b", "llama3_70b"])
    ap.add_argument("--layers", type=int, default=None)
    ap.add_argument("--compression", default="none", choices=["none", "hsz1"])
    ap.add_argument("--concurrency", type=int, default=16)
    ap.add_argument("--part-mb", type=int, default=32)
    ap.add_argument("--iters", type=int, default=2)
    ap.add_argument("--share-of", type=int, default=None,
                    help="save ONE rank's share of the model at this world size (each "
                         "parameter's dim-0 shard as a DTensor, as benchmarks/rank_share "
                         "builds it): BASELINE config 5's Llama-3-70B share on one GPU")
    args = ap.parse_args()
    rank, ws, dev = init_dist()
    from torch.distributed.device_mesh import init_device_mesh

    cfg = getattr(LlamaConfig, args.model)()
    if args.layers:
        cfg.n_layers = args.layers
    mesh = init_device_mesh(dev.type, (ws,))
    if args.share_of:
        from torch.distributed.tensor import DTensor, Shard

        from hipsnapshot import StateDict
        from hipsnapshot.models.llama import Llama

        with torch.device("meta"):
            meta = Llama(cfg)
        gen = torch.Generator(device=dev).manual_seed(0)
        params = {}
        for name, p in meta.named_parameters():
            rows = -(-p.shape[0] // args.share_of)
            local = (torch.randn((rows,) + tuple(p.shape[1:]), device=dev, generator=gen)
                     * 0.02).to(torch.bfloat16)
            params[name] = DTensor.from_local(local, mesh, [Shard(0)], run_check=False)
        del meta
        model = StateDict(**params)
        tensors = list(params.values())
    else:
        model = build_fsdp_llama(cfg, dev, torch.bfloat16, mesh=mesh)
        tensors = None
    # after a restore, compare what the state holds NOW (a StateDict's entries
    # may be re-pointed by load_state_dict)
    local_of = ((lambda: list(model.values())) if tensors is not None
                else (lambda: list(model.parameters())))
    nbytes = sum(p._local_tensor.numel() * 2 for p in local_of())
    t = torch.tensor([nbytes], dtype=torch.int64, device=dev)
    dist.all_reduce(t)
    total_bytes = int(t.item())
    srv = FakeS3Process() if rank == 0 else None
    url = [srv.url if srv else None]
    dist.broadcast_object_list(url, src=0)
    opts = {"aws_access_key_id": "AKIDFAKE", "aws_secret_access_key": "fake-secret",
            "endpoint_url": url[0], "multipart_threshold": 64 << 20,
            "part_size": args.part_mb << 20, "max_concurrency": args.concurrency}
    app = {"model": model}
    res = {"unblock_ms": [], "write_GBps": [], "restore_GBps": []}
    ok = True
    for i in range(args.iters):
        path = f"s3://ckpt/llama/step{i}"
        sync(dev)
        t0 = time.perf_counter()
        pending = Snapshot.async_take(path, app, storage_options=opts,
                                      compression=args.compression)
        tu = time.perf_counter() - t0
        pending.wait()
        tw = time.perf_counter() - t0
        tu, tw = max_over_ranks(tu, dev), max_over_ranks(tw, dev)
        res["unblock_ms"].append(round(tu * 1e3, 2))
        res["write_GBps"].append(round(total_bytes / tw / 1e9, 2))
        log(f"async_take {i}: unblock {tu * 1e3:.1f} ms, committed after {tw:.2f} s "
            f"({total_bytes / tw / 1e9:.2f} GB/s)")
        refs = [p._local_tensor.detach().clone() for p in local_of()]
        with torch.no_grad():
            for p in local_of():
                p._local_tensor.zero_()
        sync(dev)
        t0 = time.perf_counter()
        Snapshot(path, storage_options=opts).restore(app)
        sync(dev)
        tr = max_over_ranks(time.perf_counter() - t0, dev)
        res["restore_GBps"].append(round(total_bytes / tr / 1e9, 2))
        ok = ok and all(torch.equal(r, p._local_tensor) for r, p in zip(refs, local_of()))
        del refs
        log(f"restore {i}: {tr:.2f} s ({total_bytes / tr / 1e9:.2f} GB/s) bitwise ok={ok}")
    flag = torch.tensor([int(ok)], device=dev)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    emit({"bench": "async_take_s3", "model": args.model, "layers": cfg.n_layers,
          "share_of": args.share_of,
          "world_size": ws, "bytes": total_bytes, "compression": args.compression,
          "server": "fake S3, own process, loopback", "concurrency": args.concurrency,
          "part_mb": args.part_mb, **res, "restore_bitwise_ok": bool(flag.item())})
    sync(dev)
    if srv:
        srv.stop()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
