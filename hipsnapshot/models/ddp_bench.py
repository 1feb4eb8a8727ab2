"""The reference's DDP benchmark model: N fp32 parameters of ``param_mb`` MB.

Reference: `/root/reference/benchmarks/ddp/main.py:18-27,38-39` -- 200 x 100 MB
fp32 parameters (20 GB, decimal), saved with ``replicated=["**"]``.
"""

from __future__ import annotations

import torch
import torch.nn as nn


class ManyParams(nn.Module):
    def __init__(self, n_params: int = 200, param_mb: int = 100,
                 device: torch.device = torch.device("cpu")) -> None:
        super().__init__()
        numel = param_mb * 1000 * 1000 // 4
        self.params = nn.ParameterList(
            nn.Parameter(torch.empty(numel, device=device).normal_()) for _ in range(n_params))

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return sum(p[: x.numel()].dot(x) for p in self.params)
