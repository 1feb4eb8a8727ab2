"""ZeRO-3 (DeepSpeed stage 3) partitioned training state, emulated for benchmarks.

DeepSpeed is not installed here, so this module builds the state a
``DeepSpeedZeroOptimizer_Stage3`` holds on one rank for a given model shape
and exposes it through the same duck-typed surface that
``hipsnapshot.tricks.deepspeed`` patches:

* ``fp16`` flat parameter partition (what ``deepspeed.zero.Init`` keeps per rank);
* fp32 master partition(s) split into sub-groups of ``sub_group_size``
  elements (DeepSpeed's default 1e9);
* Adam ``exp_avg`` / ``exp_avg_sq`` per sub-group.

Reference benchmark: `/root/reference/benchmarks/deepspeed_opt/main.py:27-79`
(OPT, 48 layers, hidden 7168, 56 heads, fp16, ZeRO-3 Adam).  Every tensor
lives in HBM on the rank's device (288 GB per MI355X holds a 1/8 partition of
the 30B-parameter config with room to spare).
"""

from __future__ import annotations

from dataclasses import dataclass
from typing import Any, Dict, List

import torch


@dataclass
class OPTShape:
    num_hidden_layers: int = 48
    hidden_size: int = 7168
    num_attention_heads: int = 56
    vocab_size: int = 50272
    max_position_embeddings: int = 2048
    ffn_mult: int = 4

    def num_params(self) -> int:
        h, f = self.hidden_size, self.hidden_size * self.ffn_mult
        per_layer = 4 * h * h + 4 * h + 2 * h * f + f + h + 4 * h  # attn, mlp, 2 LNs
        emb = self.vocab_size * h + (self.max_position_embeddings + 2) * h
        return self.num_hidden_layers * per_layer + emb + 2 * h


def _partition(n: int, rank: int, world: int) -> int:
    per = (n + world - 1) // world
    return max(0, min(per, n - rank * per))


class EmulatedZero3Optimizer:
    """Per-rank ZeRO-3 optimizer state with DeepSpeed's ``state_dict`` layout."""

    def __init__(self, shape: OPTShape, rank: int, world_size: int, device: torch.device,
                 sub_group_size: int = 1_000_000_000, seed: int = 0) -> None:
        self.shape = shape
        self.partition_numel = _partition(shape.num_params(), rank, world_size)
        g = torch.Generator(device=device).manual_seed(seed + rank)
        self.fp16_partition = torch.empty(self.partition_numel, dtype=torch.float16,
                                          device=device)
        self.fp16_partition.normal_(0, 0.02, generator=g)
        self.fp32_groups: List[torch.Tensor] = []
        self.exp_avg: List[torch.Tensor] = []
        self.exp_avg_sq: List[torch.Tensor] = []
        left = self.partition_numel
        while left > 0:
            n = min(sub_group_size, left)
            off = self.partition_numel - left
            self.fp32_groups.append(self.fp16_partition[off:off + n].float())
            self.exp_avg.append(torch.empty(n, device=device).normal_(0, 1e-3, generator=g))
            self.exp_avg_sq.append(torch.empty(n, device=device).uniform_(0, 1e-6, generator=g))
            left -= n
        self.step = 1000
        self.persistent_parameters: List[Any] = []
        self.loaded: Dict[str, Any] = {}

    def nbytes(self) -> int:
        return self.partition_numel * (2 + 4 + 4 + 4)

    def state_dict(self) -> Dict[str, Any]:
        return {
            "zero_stage": 3,
            "loss_scaler": {"cur_scale": 65536.0, "cur_iter": self.step},
            "dynamic_loss_scale": True,
            "overflow": False,
            "partition_count": 1,
            "fp16_flat_partition": self.fp16_partition,
            "fp32_flat_groups": self.fp32_groups,
            "optimizer_state_dict": {
                "state": {i: {"step": self.step, "exp_avg": m, "exp_avg_sq": v}
                          for i, (m, v) in enumerate(zip(self.exp_avg, self.exp_avg_sq))},
                "param_groups": [{"lr": 2e-4, "weight_decay": 0.01, "betas": (0.9, 0.999),
                                  "eps": 1e-8, "params": list(range(len(self.fp32_groups)))}],
            },
        }

    def load_state_dict(self, state_dict: Dict[str, Any]) -> None:
        self._rigid_load_state_dict(state_dict)

    def _rigid_load_state_dict(self, state_dict: Dict[str, Any],
                               load_optimizer_states: bool = True) -> None:
        # in-place restore already filled our tensors; keep the scalars
        self.loaded = state_dict
        self.step = state_dict["loss_scaler"]["cur_iter"]


EmulatedZero3Optimizer.__name__ = "DeepSpeedZeroOptimizer_Stage3"


class EmulatedZero3Engine:
    """The slice of ``DeepSpeedEngine`` that the checkpoint trick touches."""

    def __init__(self, optimizer: EmulatedZero3Optimizer, rank: int) -> None:
        self.optimizer = optimizer
        self.global_rank = rank
        self.config = {"train_batch_size": 1024 ** 2, "fp16": {"enabled": True},
                       "zero_optimization": {"stage": 3},
                       "optimizer": {"type": "Adam", "params": {"lr": 2e-4,
                                                                "weight_decay": 0.01}}}

    def zero_load_from_fp32_weights(self) -> bool:
        return False
