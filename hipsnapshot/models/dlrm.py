"""DLRM-style recommendation model with row-wise sharded embedding tables.

BASELINE config 4 ("TorchRec DLRM 100GB embedding tables via uvm_tensor path").
TorchRec/fbgemm are not available, so this is a self-contained equivalent:

* ``ShardedEmbeddingBag`` -- one logical table, rows split across ranks
  (ROW_WISE), each rank's shard exposed to checkpointing as a ``DTensor``
  (``Shard(0)`` on a 1-D mesh) so snapshots are elastic like TorchRec's
  ShardedTensor tables; with ``uvm=True`` the local shard lives in managed
  memory (``hipMallocManaged``) -- the UVM path the reference stages through
  fbgemm's ``uvm_to_cpu``;
* dense bottom / top MLPs and a dot-product feature interaction.

The forward is a real (if simple) DLRM so examples can train a few steps.
"""

from __future__ import annotations

from typing import List, Optional

import torch
import torch.distributed as dist
import torch.nn as nn
import torch.nn.functional as F


class ShardedEmbeddingBag(nn.Module):
    def __init__(self, num_embeddings: int, dim: int, device: torch.device, mesh=None,
                 uvm: bool = False, dtype: torch.dtype = torch.float32) -> None:
        super().__init__()
        self.num_embeddings, self.dim = num_embeddings, dim
        ws = dist.get_world_size() if dist.is_initialized() else 1
        rank = dist.get_rank() if dist.is_initialized() else 0
        rows = (num_embeddings + ws - 1) // ws
        self.row_offset = min(rank * rows, num_embeddings)
        local_rows = max(0, min(rows, num_embeddings - self.row_offset))
        if uvm:
            from ..ops.uvm import new_managed_tensor

            local = new_managed_tensor([local_rows, dim], dtype,
                                       device.index if device.index is not None else 0)
            with torch.no_grad():
                local.uniform_(-0.01, 0.01)
        else:
            local = torch.empty(local_rows, dim, device=device, dtype=dtype).uniform_(-0.01, 0.01)
        self.mesh = mesh
        if mesh is not None:
            from torch.distributed.tensor import DTensor, Shard

            w = DTensor.from_local(local, mesh, [Shard(0)], run_check=False,
                                   shape=torch.Size([num_embeddings, dim]),
                                   stride=(dim, 1))
            self.weight = nn.Parameter(w, requires_grad=False)
        else:
            self.weight = nn.Parameter(local, requires_grad=False)

    def local_weight(self) -> torch.Tensor:
        w = self.weight
        return w._local_tensor if hasattr(w, "_local_tensor") else w

    def forward(self, ids: torch.Tensor, offsets: torch.Tensor) -> torch.Tensor:
        # single-process lookup over the local shard (ids outside it map to 0)
        local = self.local_weight()
        lid = ids - self.row_offset
        valid = (lid >= 0) & (lid < local.shape[0])
        lid = torch.where(valid, lid, torch.zeros_like(lid))
        out = F.embedding_bag(lid, local, offsets, mode="sum",
                              per_sample_weights=valid.to(local.dtype))
        if dist.is_initialized() and dist.get_world_size() > 1:
            dist.all_reduce(out)
        return out


class DLRM(nn.Module):
    def __init__(self, table_sizes: List[int], dim: int = 64, dense_in: int = 13,
                 device: Optional[torch.device] = None, mesh=None, uvm: bool = False) -> None:
        super().__init__()
        device = device or torch.device("cpu")
        self.tables = nn.ModuleList(ShardedEmbeddingBag(n, dim, device, mesh, uvm)
                                    for n in table_sizes)
        self.bottom = nn.Sequential(nn.Linear(dense_in, 128), nn.ReLU(), nn.Linear(128, dim),
                                    nn.ReLU()).to(device)
        n_feat = len(table_sizes) + 1
        self.top = nn.Sequential(nn.Linear(dim + n_feat * (n_feat - 1) // 2, 256), nn.ReLU(),
                                 nn.Linear(256, 1)).to(device)

    def forward(self, dense: torch.Tensor, sparse: List[tuple]) -> torch.Tensor:
        x = self.bottom(dense)
        feats = [x] + [t(ids, offs) for t, (ids, offs) in zip(self.tables, sparse)]
        z = torch.stack(feats, dim=1)
        inter = torch.bmm(z, z.transpose(1, 2))
        iu = torch.triu_indices(z.shape[1], z.shape[1], offset=1, device=z.device)
        flat = inter[:, iu[0], iu[1]]
        return self.top(torch.cat([x, flat], dim=1))
