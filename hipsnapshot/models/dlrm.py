"""DLRM-style recommendation model with ROW / COLUMN / TABLE-wise sharded tables.

BASELINE config 4 ("TorchRec DLRM 100GB embedding tables via uvm_tensor path").
TorchRec/fbgemm are not available, so this is a self-contained equivalent of
the layouts TorchRec's ``DistributedModelParallel`` produces (the reference
tests all three, `/root/reference/tests/gpu_tests/test_torchrec.py:181-304`):

* ``ShardedEmbeddingBag`` -- one logical table exposed to checkpointing as a
  ``DTensor``:
    - ``row``    -- ``Shard(0)`` over all ranks (ROW_WISE);
    - ``column`` -- ``Shard(1)`` over all ranks (COLUMN_WISE: every rank holds
      all rows of a slice of the embedding dim);
    - ``table``  -- the whole table on ONE rank (TABLE_WISE), a ``DTensor``
      on that rank's single-rank submesh; other ranks hold nothing of it.
  With ``uvm=True`` the local shard lives in managed memory
  (``hipMallocManaged``) -- the UVM path the reference stages through
  fbgemm's ``uvm_to_cpu``;
* dense bottom / top MLPs and a dot-product feature interaction;
* ``make_optimizer`` -- Adagrad over the tables (TorchRec's fused row-wise
  optimizer keeps the same per-table state), whose ``sum`` state has the
  table's layout.

The forward is a real (if simple) DLRM so examples can train a few steps.
"""

from __future__ import annotations

from typing import List, Optional

import torch
import torch.distributed as dist
import torch.nn as nn
import torch.nn.functional as F

SHARDINGS = ("row", "column", "table")


def _chunk(n: int, ws: int, r: int):
    """torch.chunk bounds of piece ``r`` of ``n`` split ``ws`` ways."""
    cs = (n + ws - 1) // ws
    lo = min(r * cs, n)
    return lo, min(lo + cs, n)


class ShardedEmbeddingBag(nn.Module):
    def __init__(self, num_embeddings: int, dim: int, device: torch.device, mesh=None,
                 uvm: bool = False, dtype: torch.dtype = torch.float32,
                 sharding: str = "row", owner: int = 0, submeshes=None) -> None:
        super().__init__()
        if sharding not in SHARDINGS:
            raise ValueError(f"sharding must be one of {SHARDINGS} (got {sharding!r})")
        self.num_embeddings, self.dim, self.sharding = num_embeddings, dim, sharding
        ws = dist.get_world_size() if dist.is_initialized() else 1
        rank = dist.get_rank() if dist.is_initialized() else 0
        self.owner = owner % ws
        self.row_offset, self.col_offset = 0, 0
        rows, cols = num_embeddings, dim
        if mesh is not None and sharding == "row":
            self.row_offset, hi = _chunk(num_embeddings, ws, rank)
            rows = hi - self.row_offset
        elif mesh is not None and sharding == "column":
            self.col_offset, hi = _chunk(dim, ws, rank)
            cols = hi - self.col_offset
        elif mesh is not None and sharding == "table" and rank != self.owner:
            rows = cols = 0
        if uvm and rows * cols > 0:
            from ..ops.uvm import new_managed_tensor

            local = new_managed_tensor([rows, cols], dtype,
                                       device.index if device.index is not None else 0)
            with torch.no_grad():
                local.uniform_(-0.01, 0.01)
        else:
            local = torch.empty(rows, cols, device=device, dtype=dtype).uniform_(-0.01, 0.01)
        self.mesh = mesh
        if mesh is not None:
            from torch.distributed.tensor import DTensor, Shard

            if sharding == "table":
                # a single-rank submesh per owner; every rank builds all of
                # them (group creation is collective) -- pass ``submeshes``
                # to share them between tables
                sub = (submeshes or _owner_meshes(mesh))[self.owner]
                w = DTensor.from_local(local, sub, [Shard(0)], run_check=False,
                                       shape=torch.Size([num_embeddings, dim]),
                                       stride=(dim, 1))
            else:
                w = DTensor.from_local(local, mesh, [Shard(0 if sharding == "row" else 1)],
                                       run_check=False,
                                       shape=torch.Size([num_embeddings, dim]), stride=(dim, 1))
            self.weight = nn.Parameter(w, requires_grad=False)
        else:
            self.weight = nn.Parameter(local, requires_grad=False)

    def local_weight(self) -> torch.Tensor:
        w = self.weight
        return w._local_tensor if hasattr(w, "_local_tensor") else w

    def forward(self, ids: torch.Tensor, offsets: torch.Tensor) -> torch.Tensor:
        local = self.local_weight()
        distributed = self.mesh is not None and dist.is_initialized() \
            and dist.get_world_size() > 1
        if self.sharding == "column" and distributed:
            part = F.embedding_bag(ids, local, offsets, mode="sum")
            parts = [torch.empty(part.shape[0], _chunk(self.dim, dist.get_world_size(), r)[1]
                                 - _chunk(self.dim, dist.get_world_size(), r)[0],
                                 device=part.device, dtype=part.dtype)
                     for r in range(dist.get_world_size())]
            dist.all_gather(parts, part.contiguous())
            return torch.cat(parts, dim=1)
        if self.sharding == "table" and distributed:
            out = torch.empty(offsets.numel(), self.dim, device=ids.device, dtype=local.dtype)
            if dist.get_rank() == self.owner:
                out.copy_(F.embedding_bag(ids, local, offsets, mode="sum"))
            dist.broadcast(out, src=self.owner)
            return out
        # row-wise (or unsharded): lookup over the local rows, sum over ranks
        lid = ids - self.row_offset
        valid = (lid >= 0) & (lid < local.shape[0])
        lid = torch.where(valid, lid, torch.zeros_like(lid))
        out = F.embedding_bag(lid, local, offsets, mode="sum",
                              per_sample_weights=valid.to(local.dtype))
        if distributed:
            dist.all_reduce(out)
        return out


def _owner_meshes(mesh) -> list:
    """One single-rank DeviceMesh per rank of ``mesh`` (collective: every
    rank creates every group, in the same order)."""
    from torch.distributed.device_mesh import DeviceMesh

    return [DeviceMesh(mesh.device_type, [r]) for r in mesh.mesh.flatten().tolist()]


class DLRM(nn.Module):
    def __init__(self, table_sizes: List[int], dim: int = 64, dense_in: int = 13,
                 device: Optional[torch.device] = None, mesh=None, uvm: bool = False,
                 sharding: str = "row") -> None:
        super().__init__()
        device = device or torch.device("cpu")
        subs = _owner_meshes(mesh) if mesh is not None and sharding == "table" else None
        self.tables = nn.ModuleList(
            ShardedEmbeddingBag(n, dim, device, mesh, uvm, sharding=sharding, owner=i,
                                submeshes=subs)
            for i, n in enumerate(table_sizes))
        self.bottom = nn.Sequential(nn.Linear(dense_in, 128), nn.ReLU(), nn.Linear(128, dim),
                                    nn.ReLU()).to(device)
        n_feat = len(table_sizes) + 1
        self.top = nn.Sequential(nn.Linear(dim + n_feat * (n_feat - 1) // 2, 256), nn.ReLU(),
                                 nn.Linear(256, 1)).to(device)

    def make_optimizer(self, lr: float = 0.01) -> torch.optim.Optimizer:
        """Adagrad over the embedding tables; its per-table ``sum`` state
        carries the table's sharding."""
        return torch.optim.Adagrad([t.weight for t in self.tables], lr=lr, foreach=False)

    def forward(self, dense: torch.Tensor, sparse: List[tuple]) -> torch.Tensor:
        x = self.bottom(dense)
        feats = [x] + [t(ids, offs) for t, (ids, offs) in zip(self.tables, sparse)]
        z = torch.stack(feats, dim=1)
        inter = torch.bmm(z, z.transpose(1, 2))
        iu = torch.triu_indices(z.shape[1], z.shape[1], offset=1, device=z.device)
        flat = inter[:, iu[0], iu[1]]
        return self.top(torch.cat([x, flat], dim=1))
