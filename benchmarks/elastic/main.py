#!/usr/bin/env python3
"""FSDP sharded save at N ranks, elastic restore at N/2 (BASELINE config 3, 8 -> 4).

Phase 1 (``--phase save``, N ranks) saves Llama FSDP; phase 2 (``--phase
restore``, any N') restores into a freshly sharded model and checks a few
parameters bitwise against a per-parameter checksum written at save time.
"""

import argparse
import hashlib
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from common import emit, init_dist, log, max_over_ranks, sync  # noqa: E402
from hipsnapshot import Snapshot  # noqa: E402
from hipsnapshot.models.llama import Llama, LlamaConfig, build_fsdp_llama  # noqa: E402


def checksums(model):
    """sha256 of a few full tensors, assembled on rank 0 from every rank's
    shard through CPU object collectives (works with gloo ranks that share a
    GPU, where DTensor.full_tensor() would need RCCL)."""
    from torch.distributed.tensor._utils import compute_local_shape_and_global_offset

    out = {}
    for k, v in model.state_dict().items():
        if not (k.startswith("layers.0.") or k in ("norm.weight",)):
            continue
        _, off = compute_local_shape_and_global_offset(v.shape, v.device_mesh, v.placements)
        pieces = [None] * dist.get_world_size()
        dist.all_gather_object(pieces, (list(off), v.to_local().detach().cpu()))
        if dist.get_rank() == 0:
            full = torch.empty(v.shape, dtype=v.dtype)
            for o, t in pieces:
                if t.numel():
                    full[tuple(slice(a, a + n) for a, n in zip(o, t.shape))] = t
            out[k] = hashlib.sha256(full.contiguous().view(torch.uint8).numpy().tobytes()).hexdigest()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--phase", choices=["save", "restore"], required=True)
    ap.add_argument("--path", default=os.path.join(os.environ.get("HSBENCH_DIR", "/tmp"),
                                                   "hs_elastic"))
    ap.add_argument("--model", default="llama3_8b")
    ap.add_argument("--layers", type=int, default=None)
    ap.add_argument("--backend", default=None, choices=["nccl", "gloo"],
                    help="gloo: several ranks may share one GPU (correctness rehearsal)")
    args = ap.parse_args()
    rank, ws, dev = init_dist(args.backend)
    from torch.distributed.device_mesh import init_device_mesh
    from torch.distributed.fsdp import fully_shard

    cfg = getattr(LlamaConfig, args.model)()
    if args.layers:
        cfg.n_layers = args.layers
    mesh = init_device_mesh(dev.type, (ws,))
    if args.phase == "save":
        model = build_fsdp_llama(cfg, dev, torch.bfloat16, mesh=mesh)
        sync(dev)
        t0 = time.perf_counter()
        Snapshot.take(args.path, {"model": model})
        sync(dev)
        s = max_over_ranks(time.perf_counter() - t0, dev)
        cs = checksums(model)
        if rank == 0:
            with open(args.path + ".checksums.json", "w") as f:
                json.dump(cs, f)
        nbytes = sum(p._local_tensor.numel() * 2 for p in model.parameters()) * ws
        emit({"bench": "elastic_save", "world_size": ws, "seconds": round(s, 3),
              "GBps": round(nbytes / s / 1e9, 2)})
    else:
        with torch.device("meta"):
            model = Llama(cfg).to(torch.bfloat16)
        for layer in model.layers:
            fully_shard(layer, mesh=mesh)
        fully_shard(model, mesh=mesh)
        model.to_empty(device=dev)
        sync(dev)
        t0 = time.perf_counter()
        Snapshot(args.path).restore({"model": model})
        sync(dev)
        s = max_over_ranks(time.perf_counter() - t0, dev)
        cs = checksums(model)
        ok = True
        if rank == 0:
            with open(args.path + ".checksums.json") as f:
                ref = json.load(f)
            bad = [k for k in ref if cs[k] != ref[k]]
            ok = not bad
        flag = [ok]
        dist.broadcast_object_list(flag, src=0)
        ok = flag[0]
        bad = [] if ok else ["(see rank 0)"]
        if not ok and rank == 0:
            log(f"checksum mismatch: {[k for k in ref if cs[k] != ref[k]][:5]}")
        saved_ws = Snapshot(args.path).metadata.world_size
        nbytes = sum(p._local_tensor.numel() * 2 for p in model.parameters()) * ws
        emit({"bench": "elastic_restore", "saved_world_size": saved_ws, "world_size": ws,
              "seconds": round(s, 3), "GBps": round(nbytes / s / 1e9, 2), "bitwise_ok": ok})
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
