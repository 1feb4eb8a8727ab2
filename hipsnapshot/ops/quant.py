"""Blockwise OCP-fp8 (e4m3fn) quantized save / dequantized restore (K5/K9).

Opt-in (``Snapshot.take(..., quantize=["model/**"])``): floating tensors are
written as 1 byte/element plus one fp32 scale per block of ``64*vpt``
elements (default vpt=2 -> 128-element blocks), halving bf16 checkpoint bytes
(quartering fp32).  Layout of a blob: ``[fp8 payload (n bytes, padded to 16)]
[fp32 scales]``; the entry's ``quant`` field records
``{"format": "fp8_e4m3fn_block", "block": B, "orig_dtype": ..., "payload_bytes": ...}``
and ``dtype`` stays the ORIGINAL dtype so restore targets match in place.

On a GPU the quantizer is the ``hs_fp8_quant`` HIP kernel (one wave per block,
64-lane xor-shuffle amax, ``v_cvt_pk_fp8_f32`` -- gfx950 converts to OCP
e4m3fn natively); restore runs ``hs_fp8_dequant`` on the device.  CPU tensors
use the bit-identical torch reference below (same scale rule, same RNE
conversion via ``torch.float8_e4m3fn``).
"""

from __future__ import annotations

from typing import Any, Dict

import torch

from ..format.manifest import TensorEntry
from ..format.serialization import FP8_QUANTIZABLE_DTYPES, dtype_to_string, string_to_dtype
from ..io_types import StagedBuffer

FP8_MAX = 448.0
DEFAULT_VPT = 2


def block_elems(vpt: int = DEFAULT_VPT) -> int:
    return 64 * vpt


def fp8_supported(t: torch.Tensor) -> bool:
    return t.dtype in FP8_QUANTIZABLE_DTYPES and hasattr(torch, "float8_e4m3fn") \
        and t.numel() > 0


def _layout(n: int, block: int):
    payload = (n + 15) // 16 * 16
    nblocks = (n + block - 1) // block
    return payload, nblocks, payload + 4 * nblocks


def fp8_entry_quant_info(t: torch.Tensor, vpt: int = DEFAULT_VPT) -> Dict[str, Any]:
    block = block_elems(vpt)
    payload, nblocks, total = _layout(t.numel(), block)
    return {"format": "fp8_e4m3fn_block", "block": block, "vpt": vpt,
            "orig_dtype": dtype_to_string(t.dtype), "payload_bytes": payload,
            "nblocks": nblocks, "total_bytes": total}


def quantize_reference(x: torch.Tensor, block: int):
    """Torch fp32 reference: scale = amax/448 per block (1 if amax == 0)."""
    flat = x.detach().reshape(-1).float()
    n = flat.numel()
    nblocks = (n + block - 1) // block
    padded = torch.zeros(nblocks * block, dtype=torch.float32, device=flat.device)
    padded[:n] = flat
    blocks = padded.view(nblocks, block)
    amax = blocks.abs().amax(dim=1)
    # tensor/tensor division (correctly rounded; a Python-scalar divisor is
    # lowered to a reciprocal multiply by torch and differs by 1 ulp)
    scale = torch.where(amax > 0, amax / torch.full_like(amax, FP8_MAX), torch.ones_like(amax))
    q = (blocks / scale[:, None]).clamp(-FP8_MAX, FP8_MAX).to(torch.float8_e4m3fn)
    return q.reshape(-1)[:n], scale


def dequantize_reference(q: torch.Tensor, scale: torch.Tensor, block: int,
                         dtype: torch.dtype) -> torch.Tensor:
    n = q.numel()
    nblocks = scale.numel()
    padded = torch.zeros(nblocks * block, dtype=torch.float32, device=q.device)
    padded[:n] = q.float()
    return (padded.view(nblocks, block) * scale[:, None]).reshape(-1)[:n].to(dtype)


def stage_fp8(t: torch.Tensor, entry: TensorEntry, producer: int) -> StagedBuffer:
    """Quantize ``t`` and return the blob bytes in host memory."""
    info = entry.quant
    block, vpt = info["block"], info["vpt"]
    payload, nblocks, total = info["payload_bytes"], info["nblocks"], info["total_bytes"]
    if t.is_cuda:
        from ..engine import staging
        from . import native

        dev = staging.device_of(t)
        src = t if t.is_contiguous() else t.contiguous()
        blob = torch.empty(total, dtype=torch.uint8, device=t.device)
        stream = torch.cuda.current_stream(t.device)
        if producer and producer != stream.cuda_stream:
            ev = torch.cuda.Event()
            ev.record(torch.cuda.ExternalStream(producer))
            stream.wait_event(ev)
        native.fp8_quantize(dev, src, blob[:payload], blob[payload:].view(torch.float32),
                            vpt, int(stream.cuda_stream))
        return staging.d2h_tensor(blob, int(stream.cuda_stream))
    q, scale = quantize_reference(t, block)
    blob = torch.zeros(total, dtype=torch.uint8)
    blob[: t.numel()] = q.view(torch.uint8)
    blob[payload:] = scale.view(torch.uint8)
    from ..format.serialization import contiguous_cpu_bytes_view

    return StagedBuffer(contiguous_cpu_bytes_view(blob), keepalive=blob)


def dequantize_host_fp8(buf, entry: TensorEntry) -> torch.Tensor:
    """CPU decode of an fp8 blob into a tensor of the entry's original dtype."""
    info = entry.quant
    n = 1
    for s in entry.shape:
        n *= int(s)
    mv = memoryview(buf.view if isinstance(buf, StagedBuffer) else buf).cast("B")
    raw = torch.frombuffer(bytearray(mv[: info["total_bytes"]]), dtype=torch.uint8)
    q = raw[:n].view(torch.float8_e4m3fn)
    scale = raw[info["payload_bytes"]: info["payload_bytes"] + 4 * info["nblocks"]].view(
        torch.float32)
    return dequantize_reference(q, scale, info["block"], string_to_dtype(entry.dtype)).view(
        list(entry.shape))


def dequantize_device(blob_dev: torch.Tensor, entry: TensorEntry, dst: torch.Tensor) -> None:
    """GPU decode straight into a contiguous CUDA ``dst`` of the original dtype."""
    from . import native

    info = entry.quant
    n = dst.numel()
    stream = torch.cuda.current_stream(dst.device)
    native.fp8_dequantize(dst.device.index or 0, blob_dev[:n],
                          blob_dev[info["payload_bytes"]: info["payload_bytes"]
                                   + 4 * info["nblocks"]].view(torch.float32),
                          dst, info["vpt"], int(stream.cuda_stream))
