"""Randomised fp8 quantized saves (``Snapshot.take(..., quantize=[...])``):
random shapes and float dtypes, values spanning 60 decades with zeros,
infinities and NaNs sprinkled in, every format (MX e8m0 / fp32 block /
Hadamard-rotated block), sync and async, CPU and GPU.  Every restored tensor
must equal the fp32 torch reference of its format applied to the saved
tensor -- bit for bit -- and tensors the patterns match but fp8 cannot hold
(integers) must come back losslessly.
"""

import math
import os
import random

import pytest
import torch

from hipsnapshot import Snapshot, StateDict
from hipsnapshot.ops.quant import (
    dequantize_reference,
    hadamard_dequantize_reference,
    hadamard_quantize_reference,
    mx_dequantize_reference,
    mx_quantize_reference,
    quantize_reference,
)
from hipsnapshot.utils.test_utils import env

FORMATS = ["mx", "block", "hadamard32"]


def _values(rng: random.Random, n: int, g: torch.Generator) -> torch.Tensor:
    x = torch.randn(n, generator=g, dtype=torch.float64)
    kind = rng.random()
    if kind < 0.4:
        x *= 0.02
    elif kind < 0.7:  # per-element magnitudes over many decades
        x *= torch.pow(10.0, torch.randint(-30, 30, (n,), generator=g).double())
    if rng.random() < 0.3 and n > 3:
        idx = torch.randint(0, n, (max(1, n // 50),), generator=g)
        x[idx] = rng.choice([0.0, float("inf"), float("-inf"), float("nan"), 1e-45])
    return x


def _reference(x: torch.Tensor, quant: dict) -> torch.Tensor:
    """What the restore must produce for ``x`` saved with ``quant``."""
    if quant["format"] == "fp8_e4m3fn_mx":
        q, s = mx_quantize_reference(x)
        return mx_dequantize_reference(q, s, x.dtype).view_as(x)
    if quant.get("rotation") == "hadamard32":
        q, s = hadamard_quantize_reference(x, quant["block"])
        return hadamard_dequantize_reference(q, s, x.numel(), x.dtype,
                                             quant["block"]).view_as(x)
    q, s = quantize_reference(x, quant["block"])
    return dequantize_reference(q, s, quant["block"], x.dtype).view_as(x)


def _mfma_close(got: torch.Tensor, ref: torch.Tensor, x: torch.Tensor, quant: dict) -> bool:
    """16-bit Hadamard saves on the GPU rotate on the 16-bit MFMA, which sums
    in its own order: a rotated value can differ from the k-ordered fp32
    reference in its last bit, and an fp8 code next to a rounding boundary
    then moves by one step (``csrc/hsgpu.hip`` hs_fp8_hadamard_quant16).
    Bound: NaNs in the same places, every value within 2 block scales, and
    few values off at all."""
    fmax = torch.finfo(got.dtype).max
    got, ref = got.cpu().float().reshape(-1), ref.float().reshape(-1)
    if not torch.equal(torch.isnan(got), torch.isnan(ref)):
        return False
    # a value next to fp16's largest finite one may round to inf on one side
    got, ref = got.clamp(-fmax, fmax), ref.clamp(-fmax, fmax)
    _q, s = hadamard_quantize_reference(x, quant["block"])
    per = s.repeat_interleave(quant["block"])[: got.numel()]
    ok = ~torch.isnan(ref)
    diff = (got - ref).abs()[ok]
    # (a last-bit change of the block's scale moves every value a little)
    # (one moved code shifts the 32 values of its row)
    moved = int((diff > per[ok] * 2 ** -10).sum())
    return bool((diff <= 2 * per[ok]).all() and (moved <= 64 or moved <= 0.1 * diff.numel()))


def _same(a: torch.Tensor, b: torch.Tensor) -> bool:
    """Bitwise equality with NaN == NaN."""
    a, b = a.cpu(), b.cpu()
    nan = torch.isnan(a.float())
    return bool(torch.equal(nan, torch.isnan(b.float()))
                and torch.equal(a[~nan], b[~nan]))


def _round_trip(tmp_path, seed: int, device: str) -> None:
    rng = random.Random(seed)
    g = torch.Generator().manual_seed(seed)
    fmt = rng.choice(FORMATS)
    state = {}
    for i in range(rng.randint(1, 5)):
        dtype = rng.choice([torch.float32, torch.bfloat16, torch.float16])
        n = rng.choice([1, 31, 32, 33, 127, 129, 4096, rng.randint(1, 300_000)])
        shape = [n] if rng.random() < 0.5 or n < 4 else [n // 2, 2]
        x = _values(rng, math.prod(shape), g).view(shape)
        if dtype == torch.float16:
            x = x.clamp(-6e4, 6e4)  # finite in fp16 (inf only where placed)
        state[f"w{i}"] = x.to(dtype).to(device)
    state["ids"] = torch.randint(0, 1 << 40, (rng.randint(1, 100),), generator=g).to(device)
    use_async = rng.random() < 0.4
    path = os.path.join(str(tmp_path), f"q{seed}")
    with env(HIPSNAPSHOT_FP8_FORMAT=fmt):
        app = {"sd": StateDict(**state)}
        if use_async:
            Snapshot.async_take(path, app, quantize=["sd/**"]).wait()
        else:
            Snapshot.take(path, app, quantize=["sd/**"])
    snap = Snapshot(path)
    man = snap.get_manifest()
    out = StateDict(**{k: torch.zeros_like(v) for k, v in state.items()})
    snap.restore({"sd": out})
    case = (seed, fmt, use_async, device)
    assert torch.equal(out["ids"], state["ids"]), case  # not quantizable: lossless
    for k, v in state.items():
        if k == "ids":
            continue
        quant = man[f"0/sd/{k}"].quant
        assert quant, (case, k)
        ref = _reference(v.cpu(), quant)
        check = _same
        if device != "cpu" and quant.get("rotation") == "hadamard32" and v.element_size() == 2:
            def check(a, b, v=v, quant=quant):
                return _mfma_close(a, b, v.cpu(), quant)
        assert check(out[k], ref), (case, k, v.dtype, tuple(v.shape), quant["format"])
        got = snap.read_object(f"0/sd/{k}")
        assert check(got, ref), (case, k, "read_object")


@pytest.mark.parametrize("seed", range(int(os.environ.get("HS_QUANT_SEEDS", "12"))))
def test_random_fp8_saves_match_the_reference_cpu(tmp_path, seed):
    _round_trip(tmp_path, seed, "cpu")


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(100, 100 + int(os.environ.get("HS_QUANT_SEEDS", "12"))))
def test_random_fp8_saves_match_the_reference_gpu(tmp_path, gpu, seed):
    _round_trip(tmp_path, seed, "cuda:0")


def _nonfinite_case(tmp_path, device: str, fmt: str) -> None:
    """One inf and one nan in a block: the block's other values keep their
    precision (the scale comes from the finite values), the two come back
    as NaN -- on the CPU reference path and from the GPU kernels alike (found
    by the random test: the fp32-scale formats turned the whole block into
    NaN on the CPU and into other values on the GPU)."""
    x = torch.linspace(-1.0, 1.0, 256)
    x[5], x[130] = float("inf"), float("nan")
    with env(HIPSNAPSHOT_FP8_FORMAT=fmt):
        Snapshot.take(str(tmp_path / fmt), {"sd": StateDict(w=x.to(device))}, quantize=["sd/**"])
    out = torch.zeros(256, device=device)
    Snapshot(str(tmp_path / fmt)).restore({"sd": StateDict(w=out)})
    out = out.cpu()
    nan = torch.isnan(out)
    if fmt == "hadamard32":  # a non-finite input spoils its own rotated row of 32
        assert nan[0:32].all() and nan[128:160].all() and not nan[32:128].any()
        ok = ~nan
    else:
        assert nan.nonzero().flatten().tolist() == [5, 130]
        ok = ~nan
    assert ((out[ok] - x[ok]).abs() <= 1.0 / 16).all()  # e4m3 of values <= 1


@pytest.mark.parametrize("fmt", FORMATS)
def test_nonfinite_values_do_not_spoil_their_block_cpu(tmp_path, fmt):
    _nonfinite_case(tmp_path, "cpu", fmt)


@pytest.mark.gpu
@pytest.mark.parametrize("fmt", FORMATS)
def test_nonfinite_values_do_not_spoil_their_block_gpu(tmp_path, gpu, fmt):
    _nonfinite_case(tmp_path, "cuda:0", fmt)
