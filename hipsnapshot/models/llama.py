"""Llama-3 architecture (random init) used by the benchmarks and the smoke test.

BASELINE.json's headline config is "Llama-3-8B FSDP": hidden 4096, 32 layers,
32 query heads / 8 KV heads (GQA), SwiGLU FFN 14336, vocab 128256, RMSNorm,
RoPE theta 500000, untied embeddings -> 8.03 B parameters (16.06 GB in bf16).
Only the parameter shapes matter to a checkpoint benchmark, but the module is
a complete model (forward/backward run in ``smoke()``).

``build_fsdp_llama`` materialises the model directly sharded with FSDP2
(``fully_shard`` per block + root) so every rank only ever allocates its 1/N
shard in HBM: construction on the meta device, ``to_empty`` on the rank's
GPU, then in-place random init.
"""

from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F


@dataclass
class LlamaConfig:
    vocab_size: int = 128256
    dim: int = 4096
    n_layers: int = 32
    n_heads: int = 32
    n_kv_heads: int = 8
    ffn_dim: int = 14336
    norm_eps: float = 1e-5
    rope_theta: float = 500000.0
    max_seq_len: int = 8192

    @classmethod
    def llama3_8b(cls) -> "LlamaConfig":
        return cls()

    @classmethod
    def llama3_70b(cls) -> "LlamaConfig":
        return cls(dim=8192, n_layers=80, n_heads=64, n_kv_heads=8, ffn_dim=28672)

    @classmethod
    def tiny(cls) -> "LlamaConfig":
        return cls(vocab_size=512, dim=128, n_layers=2, n_heads=4, n_kv_heads=2, ffn_dim=256,
                   max_seq_len=128)

    def num_params(self) -> int:
        hd = self.dim // self.n_heads
        attn = self.dim * (self.n_heads * hd) + 2 * self.dim * (self.n_kv_heads * hd) \
            + (self.n_heads * hd) * self.dim
        mlp = 3 * self.dim * self.ffn_dim
        per_layer = attn + mlp + 2 * self.dim
        return self.n_layers * per_layer + 2 * self.vocab_size * self.dim + self.dim


class RMSNorm(nn.Module):
    def __init__(self, dim: int, eps: float) -> None:
        super().__init__()
        self.eps = eps
        self.weight = nn.Parameter(torch.ones(dim))

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        xf = x.float()
        y = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + self.eps)
        return y.type_as(x) * self.weight


def rope_tables(head_dim: int, seq_len: int, theta: float, device) -> tuple:
    inv = 1.0 / (theta ** (torch.arange(0, head_dim, 2, device=device).float() / head_dim))
    t = torch.arange(seq_len, device=device).float()
    freqs = torch.outer(t, inv)
    return freqs.cos(), freqs.sin()


def apply_rope(x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor) -> torch.Tensor:
    x1, x2 = x[..., 0::2].float(), x[..., 1::2].float()
    c, s = cos[None, :, None, :], sin[None, :, None, :]
    out = torch.stack((x1 * c - x2 * s, x1 * s + x2 * c), dim=-1).flatten(-2)
    return out.type_as(x)


class Attention(nn.Module):
    def __init__(self, cfg: LlamaConfig) -> None:
        super().__init__()
        self.n_heads, self.n_kv = cfg.n_heads, cfg.n_kv_heads
        self.hd = cfg.dim // cfg.n_heads
        self.wq = nn.Linear(cfg.dim, cfg.n_heads * self.hd, bias=False)
        self.wk = nn.Linear(cfg.dim, cfg.n_kv_heads * self.hd, bias=False)
        self.wv = nn.Linear(cfg.dim, cfg.n_kv_heads * self.hd, bias=False)
        self.wo = nn.Linear(cfg.n_heads * self.hd, cfg.dim, bias=False)

    def forward(self, x, cos, sin):
        b, s, _ = x.shape
        q = self.wq(x).view(b, s, self.n_heads, self.hd)
        k = self.wk(x).view(b, s, self.n_kv, self.hd)
        v = self.wv(x).view(b, s, self.n_kv, self.hd)
        q, k = apply_rope(q, cos, sin), apply_rope(k, cos, sin)
        rep = self.n_heads // self.n_kv
        k = k.repeat_interleave(rep, dim=2)
        v = v.repeat_interleave(rep, dim=2)
        o = F.scaled_dot_product_attention(q.transpose(1, 2), k.transpose(1, 2),
                                           v.transpose(1, 2), is_causal=True)
        return self.wo(o.transpose(1, 2).reshape(b, s, -1))


class FeedForward(nn.Module):
    def __init__(self, cfg: LlamaConfig) -> None:
        super().__init__()
        self.w1 = nn.Linear(cfg.dim, cfg.ffn_dim, bias=False)
        self.w2 = nn.Linear(cfg.ffn_dim, cfg.dim, bias=False)
        self.w3 = nn.Linear(cfg.dim, cfg.ffn_dim, bias=False)

    def forward(self, x):
        return self.w2(F.silu(self.w1(x)) * self.w3(x))


class Block(nn.Module):
    def __init__(self, cfg: LlamaConfig) -> None:
        super().__init__()
        self.attention_norm = RMSNorm(cfg.dim, cfg.norm_eps)
        self.attention = Attention(cfg)
        self.ffn_norm = RMSNorm(cfg.dim, cfg.norm_eps)
        self.feed_forward = FeedForward(cfg)

    def forward(self, x, cos, sin):
        h = x + self.attention(self.attention_norm(x), cos, sin)
        return h + self.feed_forward(self.ffn_norm(h))


class Llama(nn.Module):
    def __init__(self, cfg: LlamaConfig) -> None:
        super().__init__()
        self.cfg = cfg
        self.tok_embeddings = nn.Embedding(cfg.vocab_size, cfg.dim)
        self.layers = nn.ModuleList(Block(cfg) for _ in range(cfg.n_layers))
        self.norm = RMSNorm(cfg.dim, cfg.norm_eps)
        self.output = nn.Linear(cfg.dim, cfg.vocab_size, bias=False)

    def forward(self, tokens: torch.Tensor) -> torch.Tensor:
        s = tokens.shape[1]
        hd = self.cfg.dim // self.cfg.n_heads
        cos, sin = rope_tables(hd, s, self.cfg.rope_theta, tokens.device)
        h = self.tok_embeddings(tokens)
        for layer in self.layers:
            h = layer(h, cos, sin)
        return self.output(self.norm(h))


@torch.no_grad()
def init_weights_(model: nn.Module, std: float = 0.02, seed: Optional[int] = 0) -> None:
    """Random init in place (works on DTensor params: each rank fills its shard)."""
    gen = None
    for name, p in model.named_parameters():
        local = p._local_tensor if hasattr(p, "_local_tensor") else p
        if name.endswith("norm.weight") or "_norm" in name:
            local.fill_(1.0)
        else:
            if gen is None or gen.device != local.device:
                gen = torch.Generator(device=local.device)
                if seed is not None:
                    gen.manual_seed(seed + (torch.distributed.get_rank()
                                            if torch.distributed.is_initialized() else 0))
            local.normal_(0.0, std, generator=gen)


def build_fsdp_llama(cfg: LlamaConfig, device: torch.device,
                     dtype: torch.dtype = torch.bfloat16, mesh=None,
                     compute_dtype: Optional[torch.dtype] = None) -> nn.Module:
    """Llama sharded with FSDP2 (DTensor params, Shard(0)) on ``mesh``.

    ``dtype`` is the stored (master) parameter dtype; a different
    ``compute_dtype`` (e.g. fp32 master weights, bf16 compute) installs an
    FSDP2 mixed-precision policy with fp32 gradient reduction.
    """
    from torch.distributed.fsdp import fully_shard

    with torch.device("meta"):
        model = Llama(cfg).to(dtype)
    kw = {"mesh": mesh} if mesh is not None else {}
    if compute_dtype is not None and compute_dtype != dtype:
        from torch.distributed.fsdp import MixedPrecisionPolicy

        kw["mp_policy"] = MixedPrecisionPolicy(param_dtype=compute_dtype,
                                               reduce_dtype=torch.float32)
    for layer in model.layers:
        fully_shard(layer, **kw)
    fully_shard(model, **kw)
    model.to_empty(device=device)
    init_weights_(model, std=1.0 / math.sqrt(cfg.dim))
    return model


def llama_tp_plan(model: "Llama") -> dict:
    """Megatron-style tensor-parallel plan: column-wise q/k/v/w1/w3 and the
    output head, row-wise wo/w2 and the token embedding."""
    from torch.distributed.tensor.parallel import ColwiseParallel, RowwiseParallel

    plan = {"tok_embeddings": RowwiseParallel(), "output": ColwiseParallel()}
    for i in range(len(model.layers)):
        for n in ("attention.wq", "attention.wk", "attention.wv", "feed_forward.w1",
                  "feed_forward.w3"):
            plan[f"layers.{i}.{n}"] = ColwiseParallel()
        for n in ("attention.wo", "feed_forward.w2"):
            plan[f"layers.{i}.{n}"] = RowwiseParallel()
    return plan


def build_2d_llama(cfg: LlamaConfig, device: torch.device, mesh,
                   dtype: torch.dtype = torch.bfloat16, tp_dim: str = "tp",
                   dp_dim: str = "dp") -> nn.Module:
    """Llama with tensor parallelism on ``mesh[tp_dim]`` and FSDP2 on
    ``mesh[dp_dim]`` (2-D parallel).  Parameters that TP already split on dim
    0 carry ``(_StridedShard(0), Shard(0))`` placements; row-wise ones carry
    ``(Shard(0), Shard(1))``; norms ``(Shard(0), Replicate())``."""
    from torch.distributed.fsdp import fully_shard
    from torch.distributed.tensor.parallel import parallelize_module

    with torch.device("meta"):
        model = Llama(cfg).to(dtype)
    tp = mesh[tp_dim]
    parallelize_module(model, tp, llama_tp_plan(model))
    for layer in model.layers:  # local head counts after the column split
        layer.attention.n_heads //= tp.size()
        layer.attention.n_kv //= tp.size()
    for layer in model.layers:
        fully_shard(layer, mesh=mesh[dp_dim])
    fully_shard(model, mesh=mesh[dp_dim])
    model.to_empty(device=device)
    init_weights_(model, std=1.0 / math.sqrt(cfg.dim))
    return model
