"""Blockwise OCP-fp8 (e4m3fn) quantized save / dequantized restore (K5/K9).

Opt-in (``Snapshot.take(..., quantize=["model/**"])``): floating tensors are
written as 1 byte/element plus one fp32 scale per 128-element block, halving
bf16 checkpoint bytes (quartering fp32).  The entry's ``dtype`` stays the
ORIGINAL dtype so restore targets match in place; ``quant`` records the
layout::

    {"format": "fp8_e4m3fn_block", "block": 128, "rotation": "hadamard32"|"none",
     "payload_bytes": P, "nblocks": B, "total_bytes": P + 4B, ...}

blob = ``[fp8 payload (P bytes)][B fp32 scales]``.

rotation ``"hadamard32"`` (opt-in, ``HIPSNAPSHOT_FP8_FORMAT=hadamard32``): the flat
tensor is cut into groups of 32 elements and each group is multiplied by the
32x32 Sylvester Hadamard matrix H (+-1 entries) before quantization; restore
computes ``(Y' H) / 32``.  The rotation spreads outliers over the group; for
e4m3 that only pays when a block's dynamic range exceeds the format's (see
``default_rotation``), so it is off by default.  On MI355X both directions run on the
matrix cores.  bf16 / f16 tensors are rotated by ``v_mfma_f32_32x32x16_{bf16,f16}``
(``hs_fp8_hadamard_quant16``: 2 MFMAs per 1024 elements; the MFMA sums 16 exact
products in its own order, so a code can differ from the fp32 reference by one
fp8 ulp -- tests bound it.  So a bf16 / f16 tensor's rotated blob is NOT
byte-reproducible across devices: quantized on the GPU and on the CPU it can
give different codes, blob bytes and checksums.  Nothing depends on the two
matching -- a checksum is of the bytes actually written, and replicated
entries are deduplicated by manifest, not by blob contents); fp32 tensors use ``v_mfma_f32_32x32x2_f32``
(exact f32 k-ordered FMA chains, ``hs_fp8_hadamard_quant``), bit-identical to
the torch reference below, which uses the same sequential k order.  Every
dequantization runs on ``v_mfma_f32_32x32x16_bf16`` over the codes widened to
bf16 (``hs_fp8_hadamard_dequant8``): the row sums of e4m3 values are exact, so
GPU and torch restores agree bit for bit.

rotation ``"none"`` (default): plain blockwise quantization (``hs_fp8_quant`` kernel:
one wave per block, 64-lane xor-shuffle amax, ``v_cvt_pk_fp8_f32`` -- gfx950
converts to OCP e4m3fn natively).

Scale rule (both): ``scale = amax / 448`` (correctly rounded; 1 when the block
is all zeros), ``q = e4m3fn(clamp(y / scale))`` with round-to-nearest-even.

MX layout (default for un-rotated tensors; ``HIPSNAPSHOT_FP8_FORMAT=block``
selects the fp32-scale layout above)::

    {"format": "fp8_e4m3fn_mx", "block": 32, "scale": "e8m0", "rotation": "none",
     "payload_bytes": P = round_up(n, 16), "nblocks": B = ceil(n / 32),
     "total_bytes": P + B}

blob = ``[fp8 payload (P bytes, zero padded)][B E8M0 scale bytes]`` -- the OCP
MX block format: one power-of-two scale ``2^k`` per 32 elements, byte
``k + 127``.  ``k`` is the smallest exponent with ``amax <= 448 * 2^k``
(``amax`` over the block's finite elements; inf / nan are stored as e4m3fn
NaN with their sign, as torch's cast does)
(``amax = m * 2^e`` by frexp: ``k = e - 9`` if ``m <= 0.875`` else ``e - 8``;
0 for all-zero / non-finite blocks, clamped to [-127, 127]), so ``x * 2^-k``
is EXACT: no division, no saturation, and restore ``q * 2^k`` is exact in
fp32.  That takes the per-element correctly rounded division off the GPU
(``hs_mx8_quant`` streams at the HBM roof) while the blob stays bit-identical
to the torch reference below.  Same 1/32 scale overhead as fp32 scales per
128 elements, at 4x finer granularity.
"""

from __future__ import annotations

import os
from typing import Any, Dict

import torch

from ..format.manifest import TensorEntry
from ..format.serialization import FP8_QUANTIZABLE_DTYPES, dtype_to_string, string_to_dtype
from ..io_types import StagedBuffer

FP8_MAX = 448.0
DEFAULT_VPT = 2
GROUP = 32


def block_elems(vpt: int = DEFAULT_VPT) -> int:
    return 64 * vpt


def default_rotation() -> str:
    # Measured (tests/test_quant.py::test_rotation_error_tradeoff): e4m3 is a
    # floating format, so an outlier only costs its own relative precision;
    # rotating spreads the outlier's absolute error over its whole group.  On
    # Student-t(2) weights the rotated L2 error is ~1.6x the plain one, so the
    # rotation is opt-in; it pays when a block's dynamic range exceeds e4m3's
    # ~2^15 (values far below amax would otherwise fall into subnormals).
    from .. import knobs

    return "hadamard32" if knobs.fp8_format() == "hadamard32" else "none"


def default_scale() -> str:
    """``e8m0`` (MX, default) or ``fp32`` (``HIPSNAPSHOT_FP8_FORMAT=block``)
    for un-rotated quantization."""
    from .. import knobs

    return "fp32" if knobs.fp8_format() == "block" else "e8m0"


MX_BLOCK = 32


def is_mx(info: Dict[str, Any]) -> bool:
    return info.get("format") == "fp8_e4m3fn_mx"


def fp8_supported(t: torch.Tensor) -> bool:
    return t.dtype in FP8_QUANTIZABLE_DTYPES and hasattr(torch, "float8_e4m3fn") \
        and t.numel() > 0


def _round_up(n: int, m: int) -> int:
    return (n + m - 1) // m * m


def fp8_entry_quant_info(t: torch.Tensor, vpt: int = DEFAULT_VPT,
                         rotation: str = None) -> Dict[str, Any]:
    rotation = rotation or default_rotation()
    n = t.numel()
    if rotation == "none" and default_scale() == "e8m0":
        payload = _round_up(n, 16)
        nblocks = (n + MX_BLOCK - 1) // MX_BLOCK
        return {"format": "fp8_e4m3fn_mx", "block": MX_BLOCK, "scale": "e8m0",
                "rotation": "none", "orig_dtype": dtype_to_string(t.dtype),
                "payload_bytes": payload, "nblocks": nblocks, "total_bytes": payload + nblocks}
    if rotation == "hadamard32":
        block = 128
        n_q = _round_up(n, GROUP)
    else:
        block = block_elems(vpt)
        n_q = n
    payload = _round_up(n_q, 16)
    nblocks = (n_q + block - 1) // block
    return {"format": "fp8_e4m3fn_block", "block": block, "vpt": vpt, "rotation": rotation,
            "orig_dtype": dtype_to_string(t.dtype), "payload_bytes": payload,
            "nblocks": nblocks, "total_bytes": payload + 4 * nblocks}


# ---------------------------------------------------------------------------
# torch fp32 references
# ---------------------------------------------------------------------------

def _scale_and_quant(blocks: torch.Tensor):
    # over the finite elements: an inf / nan does not set its block's scale,
    # and its code is the e4m3fn NaN with its sign (torch's cast of inf / nan),
    # as in the MX format and the GPU kernels (``csrc/hsgpu.hip`` fp8_fix_nonfinite)
    finite = torch.isfinite(blocks)
    amax = torch.where(finite, blocks.abs(), torch.zeros_like(blocks)).amax(dim=1)
    # tensor/tensor division (correctly rounded; a Python-scalar divisor is
    # lowered to a reciprocal multiply by torch and differs by 1 ulp)
    scale = torch.where(amax > 0, amax / torch.full_like(amax, FP8_MAX), torch.ones_like(amax))
    # one reciprocal per block, one multiply per element (the kernels' rule)
    inv = torch.ones_like(scale) / scale
    q = torch.where(finite, (blocks * inv[:, None]).clamp(-FP8_MAX, FP8_MAX),
                    blocks).to(torch.float8_e4m3fn)
    return q, scale


def quantize_reference(x: torch.Tensor, block: int):
    """Plain blockwise reference: returns (q[n] e4m3fn, scale[nblocks])."""
    flat = x.detach().reshape(-1).float()
    n = flat.numel()
    nblocks = (n + block - 1) // block
    padded = torch.zeros(nblocks * block, dtype=torch.float32, device=flat.device)
    padded[:n] = flat
    q, scale = _scale_and_quant(padded.view(nblocks, block))
    return q.reshape(-1)[:n], scale


def dequantize_reference(q: torch.Tensor, scale: torch.Tensor, block: int,
                         dtype: torch.dtype) -> torch.Tensor:
    n = q.numel()
    nblocks = scale.numel()
    padded = torch.zeros(nblocks * block, dtype=torch.float32, device=q.device)
    padded[:n] = q.float()
    return (padded.view(nblocks, block) * scale[:, None]).reshape(-1)[:n].to(dtype)


def pow2(e: torch.Tensor) -> torch.Tensor:
    """Exact float32 ``2**e`` for integer ``e`` in [-149, 127] (bit-built:
    normal exponents, or the subnormal bit below -126)."""
    e = e.to(torch.int32)
    normal = (e + 127).clamp(min=1) << 23
    sub = torch.ones_like(e) << (e + 149).clamp(0, 22)
    return torch.where(e >= -126, normal, sub).view(torch.float32)


def mx_exponents(amax: torch.Tensor) -> torch.Tensor:
    """Per-block ``k``: smallest exponent with ``amax <= 448 * 2^k``."""
    m, e = torch.frexp(amax)
    k = torch.where(m <= 0.875, e - 9, e - 8)
    ok = (amax > 0) & torch.isfinite(amax)
    return torch.where(ok, k, torch.zeros_like(k)).clamp(-127, 127).to(torch.int32)


def mx_quantize_reference(x: torch.Tensor):
    """MX reference: returns (q[n] e4m3fn, scale bytes[nblocks] uint8)."""
    flat = x.detach().reshape(-1).float()
    n = flat.numel()
    nblocks = (n + MX_BLOCK - 1) // MX_BLOCK
    blocks = torch.zeros(nblocks * MX_BLOCK, dtype=torch.float32, device=flat.device)
    blocks[:n] = flat
    blocks = blocks.view(nblocks, MX_BLOCK)
    a = blocks.abs()
    amax = torch.where(torch.isfinite(a), a, torch.zeros_like(a)).amax(dim=1)  # finite only
    k = mx_exponents(amax)
    q = (blocks * pow2(-k)[:, None]).to(torch.float8_e4m3fn)
    return q.reshape(-1)[:n], (k + 127).to(torch.uint8)


def mx_dequantize_reference(q: torch.Tensor, sbytes: torch.Tensor,
                            dtype: torch.dtype) -> torch.Tensor:
    n = q.numel()
    nblocks = sbytes.numel()
    padded = torch.zeros(nblocks * MX_BLOCK, dtype=torch.float32, device=q.device)
    padded[:n] = q.float()
    k = sbytes.to(torch.int32) - 127
    return (padded.view(nblocks, MX_BLOCK) * pow2(k)[:, None]).reshape(-1)[:n].to(dtype)


def hadamard_matrix(n: int = GROUP, device=None) -> torch.Tensor:
    idx = torch.arange(n, device=device)
    bits = (idx[:, None] & idx[None, :])
    parity = torch.zeros_like(bits)
    for b in range(n.bit_length()):
        parity ^= (bits >> b) & 1
    return 1.0 - 2.0 * parity.float()


# k order of the GPU kernels' MFMA chain: step t contracts k = t (lanes of
# half 0) then k = 16 + t (half 1), the layout that lets each lane load its
# 16 elements of a row with 16-B vector loads (hs_fp8_hadamard_*)
HADAMARD_K_ORDER = [k for t in range(GROUP // 2) for k in (t, GROUP // 2 + t)]


def _rotate_sequential(rows: torch.Tensor) -> torch.Tensor:
    """rows[R, 32] @ H with a k-ordered fp32 FMA chain (= MFMA f32 semantics,
    in ``HADAMARD_K_ORDER``)."""
    h = hadamard_matrix(GROUP, rows.device)
    acc = torch.zeros_like(rows)
    for k in HADAMARD_K_ORDER:
        acc = acc + rows[:, k:k + 1] * h[k][None, :]  # x * +-1 is exact: one rounding
    return acc


def hadamard_quantize_reference(x: torch.Tensor, block: int = 128):
    """Returns (q[n_pad] e4m3fn, scale[nblocks]) with n_pad = round_up(n, 32)."""
    flat = x.detach().reshape(-1).float()
    n = flat.numel()
    n_pad = _round_up(n, GROUP)
    nblocks = (n_pad + block - 1) // block
    rows = torch.zeros(nblocks * block // GROUP, GROUP, dtype=torch.float32, device=flat.device)
    rows.view(-1)[:n] = flat
    y = _rotate_sequential(rows).reshape(nblocks, block)
    q, scale = _scale_and_quant(y)
    return q.reshape(-1)[:n_pad], scale


def hadamard_dequantize_reference(q: torch.Tensor, scale: torch.Tensor, n: int,
                                  dtype: torch.dtype, block: int = 128) -> torch.Tensor:
    """x = (Q H) * (s / 32): the row sums of e4m3 codes are exact (multiples of
    2^-9 below 2^14, computed in float64 and exact in fp32), then ONE fp32
    rounding by the block scale -- the same arithmetic as the GPU kernel
    (``hs_fp8_hadamard_dequant8``, bf16 MFMA on the widened codes), so both
    are bit-identical."""
    n_pad = q.numel()
    rows = q.float().reshape(-1, GROUP).double()
    h = hadamard_matrix(GROUP, rows.device).double()
    z = (rows @ h).float()  # exact
    s = (scale.float() * (1.0 / GROUP)).repeat_interleave(block // GROUP)[:z.shape[0]]
    x = z * s[:, None]
    return x.reshape(-1)[:n].to(dtype)


# ---------------------------------------------------------------------------
# staging (save) and decoding (restore)
# ---------------------------------------------------------------------------

def stage_fp8(t: torch.Tensor, entry: TensorEntry, producer: int) -> StagedBuffer:
    """Quantize ``t`` and return the blob bytes in host memory."""
    info = entry.quant
    rot = info.get("rotation", "none")
    payload, nblocks, total = info["payload_bytes"], info["nblocks"], info["total_bytes"]
    if is_mx(info):
        return _stage_mx(t, info, producer)
    if t.is_cuda:
        from ..engine import staging
        from . import native

        dev = staging.device_of(t)
        src = t if t.is_contiguous() else t.contiguous()
        blob = torch.zeros(total, dtype=torch.uint8, device=t.device)
        stream = torch.cuda.current_stream(t.device)
        if producer is not None and producer != stream.cuda_stream:
            ev = torch.cuda.Event()
            ev.record(torch.cuda.default_stream(t.device) if producer == 0
                      else torch.cuda.ExternalStream(producer))
            stream.wait_event(ev)
        scales = blob[payload:].view(torch.float32)
        if rot == "hadamard32":
            native.fp8_hadamard_quantize(dev, src, blob[:payload], scales,
                                         int(stream.cuda_stream))
        else:
            native.fp8_quantize(dev, src, blob[:payload], scales, info["vpt"],
                                int(stream.cuda_stream))
        return staging.d2h_tensor(blob, int(stream.cuda_stream))
    if rot == "hadamard32":
        q, scale = hadamard_quantize_reference(t, info["block"])
    else:
        q, scale = quantize_reference(t, info["block"])
    blob = torch.zeros(total, dtype=torch.uint8)
    blob[: q.numel()] = q.view(torch.uint8)
    blob[payload:] = scale.view(torch.uint8)
    from ..format.serialization import contiguous_cpu_bytes_view

    return StagedBuffer(contiguous_cpu_bytes_view(blob), keepalive=blob)


def _stage_mx(t: torch.Tensor, info: Dict[str, Any], producer: int) -> StagedBuffer:
    payload, total = info["payload_bytes"], info["total_bytes"]
    if t.is_cuda:
        from ..engine import staging
        from . import native

        dev = staging.device_of(t)
        stream = torch.cuda.current_stream(t.device)
        if producer is not None and producer != stream.cuda_stream:
            ev = torch.cuda.Event()
            ev.record(torch.cuda.default_stream(t.device) if producer == 0
                      else torch.cuda.ExternalStream(producer))
            stream.wait_event(ev)
        src = t if t.is_contiguous() else t.contiguous()
        blob = torch.empty(total, dtype=torch.uint8, device=t.device)  # kernel writes all of it
        native.mx8_quantize(dev, src, blob[:payload], blob[payload:], int(stream.cuda_stream))
        return staging.d2h_tensor(blob, int(stream.cuda_stream))
    q, sbytes = mx_quantize_reference(t)
    blob = torch.zeros(total, dtype=torch.uint8)
    blob[: q.numel()] = q.view(torch.uint8)
    blob[payload:] = sbytes
    from ..format.serialization import contiguous_cpu_bytes_view

    return StagedBuffer(contiguous_cpu_bytes_view(blob), keepalive=blob)


def _split_blob(raw: torch.Tensor, info: Dict[str, Any], n: int):
    rot = info.get("rotation", "none")
    nq = _round_up(n, GROUP) if rot == "hadamard32" else n
    q = raw[:nq]
    scale = raw[info["payload_bytes"]: info["payload_bytes"] + 4 * info["nblocks"]].view(
        torch.float32)
    return rot, q, scale


def dequantize_host_fp8(buf, entry: TensorEntry) -> torch.Tensor:
    """CPU decode of an fp8 blob into a tensor of the entry's original dtype."""
    info = entry.quant
    n = 1
    for s in entry.shape:
        n *= int(s)
    mv = memoryview(buf.view if isinstance(buf, StagedBuffer) else buf).cast("B")
    raw = torch.frombuffer(bytearray(mv[: info["total_bytes"]]), dtype=torch.uint8)
    dtype = string_to_dtype(entry.dtype)
    if is_mx(info):
        p = info["payload_bytes"]
        out = mx_dequantize_reference(raw[:n].view(torch.float8_e4m3fn),
                                      raw[p: p + info["nblocks"]], dtype)
        return out.view(list(entry.shape))
    rot, q, scale = _split_blob(raw, info, n)
    if rot == "hadamard32":
        out = hadamard_dequantize_reference(q.view(torch.float8_e4m3fn), scale, n, dtype,
                                            info["block"])
    else:
        out = dequantize_reference(q.view(torch.float8_e4m3fn), scale, info["block"], dtype)
    return out.view(list(entry.shape))


def dequantize_device(blob_dev: torch.Tensor, entry: TensorEntry, dst: torch.Tensor) -> None:
    """GPU decode straight into a contiguous CUDA ``dst`` of the original dtype."""
    from . import native

    info = entry.quant
    n = dst.numel()
    stream = int(torch.cuda.current_stream(dst.device).cuda_stream)
    dev = dst.device.index or 0
    if is_mx(info):
        p = info["payload_bytes"]
        native.mx8_dequantize(dev, blob_dev[:n], blob_dev[p: p + info["nblocks"]], dst, stream)
        return
    rot, q, scale = _split_blob(blob_dev, info, n)
    if rot == "hadamard32":
        native.fp8_hadamard_dequantize(dev, q, scale, dst, stream)
    else:
        native.fp8_dequantize(dev, q, scale, dst, info["vpt"], stream)
