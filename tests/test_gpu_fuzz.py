"""Randomised GPU checks of the two hand-written data-plane kernels every take
and restore runs, against PyTorch / the NumPy reference:

* ``hs_copy_nd`` (``csrc/hsgpu.hip``): batches of random strided views --
  permuted, step-sliced, narrowed, 1-4-D, same-dtype and casting, into
  contiguous or strided destinations -- each batch ONE launch, every
  destination compared with ``src.to(dst_dtype)`` (bit-exact) and the bytes
  around it checked untouched;
* the HSZ1 coder (``csrc/hsz.hip``): adversarial byte distributions (1 to 256
  distinct high bytes, skewed weights, every element width), GPU blob ==
  reference blob byte for byte, GPU decode == input.

Seeded (``random.Random``), so a failure names its case and reproduces.
"""

import random

import numpy as np
import pytest
import torch

from hipsnapshot.ops import native

pytestmark = pytest.mark.gpu

FLOATS = [torch.float32, torch.bfloat16, torch.float16, torch.float64]
INTS = [torch.uint8, torch.int16, torch.int32, torch.int64]


def _random_view(rng: random.Random, base: torch.Tensor) -> torch.Tensor:
    """A random non-overlapping view of ``base``: permute, step slices, narrow."""
    v = base.permute(*rng.sample(range(base.dim()), base.dim()))
    for d in range(v.dim()):
        n = v.shape[d]
        if n > 1 and rng.random() < 0.5:
            lo = rng.randrange(n)
            hi = rng.randrange(lo + 1, n + 1)
            step = rng.choice([1, 1, 2, 3])
            v = v.narrow(d, lo, hi - lo)[(slice(None),) * d + (slice(None, None, step),)]
    return v


def _random_case(rng: random.Random, dev):
    ndim = rng.randint(1, 4)
    big = rng.randrange(ndim) if rng.random() < 0.3 else -1
    shape = [rng.randint(1, 600 if d == big else (70 if ndim <= 2 else 24))
             for d in range(ndim)]
    if rng.random() < 0.6:
        sdt = ddt = rng.choice(FLOATS + INTS)
    else:
        sdt, ddt = rng.choice(FLOATS), rng.choice(FLOATS)
    if sdt.is_floating_point:
        base = (torch.randn(shape, device=dev, dtype=torch.float64) * 50).to(sdt)
    else:
        base = torch.randint(0, 120, shape, device=dev, dtype=torch.int64).to(sdt)
    src = _random_view(rng, base)
    if rng.random() < 0.5:
        dst_buf = torch.zeros(src.numel(), dtype=ddt, device=dev)
        dst = dst_buf.view(src.shape)
    else:
        # a strided window of a padded, permuted buffer
        perm = rng.sample(range(src.dim()), src.dim())
        pad = [src.shape[p] + rng.randint(0, 3) for p in perm]
        dst_buf = torch.zeros(pad, dtype=ddt, device=dev)
        win = dst_buf
        for d, p in enumerate(perm):
            win = win.narrow(d, pad[d] - src.shape[p], src.shape[p])
        inv = [perm.index(i) for i in range(src.dim())]
        dst = win.permute(*inv)
    return src, dst, dst_buf


def test_copy_nd_random_views_vs_torch(gpu):
    rng = random.Random(20261019)
    torch.manual_seed(0)
    stream = int(torch.cuda.current_stream().cuda_stream)
    n_cases = 0
    for batch_i in range(40):
        cases = [_random_case(rng, gpu) for _ in range(rng.randint(1, 24))]
        b = native.CopyBatch()
        for src, dst, _buf in cases:
            # host-side shape check before the launch: the kernel trusts them
            assert tuple(src.shape) == tuple(dst.shape)
            b.add(src.data_ptr(), src.dtype, src.stride(), dst.data_ptr(), dst.dtype,
                  dst.stride(), list(src.shape), src.element_size())
        b.launch(0, stream, sync=True)
        for ci, (src, dst, buf) in enumerate(cases):
            ref = src.to(dst.dtype)
            assert torch.equal(dst, ref), (batch_i, ci, tuple(src.shape), src.stride(),
                                           dst.stride(), src.dtype, dst.dtype)
            # nothing outside the destination window was written
            outside = buf.clone()
            dst_in = outside.as_strided(dst.shape, dst.stride(),
                                        dst.storage_offset() - buf.storage_offset())
            dst_in.zero_()
            assert not outside.any(), (batch_i, ci)
            n_cases += 1
    assert n_cases > 400


def _adversarial(seed: int, w: int, n: int) -> np.ndarray:
    rng = np.random.default_rng(seed)
    alphabet = int(rng.integers(1, 257))
    skew = float(rng.uniform(0.0, 3.0))
    p = np.arange(1, alphabet + 1, dtype=np.float64) ** -skew
    vals = rng.permutation(256)[:alphabet].astype(np.uint8)
    raw = rng.integers(0, 256, size=n, dtype=np.uint8)
    hi = vals[rng.choice(alphabet, size=n, p=p / p.sum())]
    if w > 1:
        raw[w - 1::w] = hi[w - 1::w]
    else:
        raw[:] = hi
    return raw


@pytest.mark.parametrize("w", [1, 2, 4, 8])
def test_hsz_gpu_adversarial_distributions(gpu, w):
    from hipsnapshot.ops import codec

    s = torch.cuda.current_stream()
    rng = random.Random(w)
    for case in range(20):
        n = rng.choice([rng.randint(1, 5000), rng.randint(60_000, 300_000)])
        frame = rng.choice([16 * 1024, 64 * 1024])
        raw = _adversarial(1000 * w + case, w, n)
        ref = codec.encode_cpu(raw, w, frame, nthreads=4).tobytes()  # == the NumPy reference
        d = torch.from_numpy(raw).to(gpu)
        out, total, _ = codec.encode_device(d, w, int(s.cuda_stream), frame)
        s.synchronize()
        nb = int(total.item())
        assert nb == len(ref), (w, case, n, frame)
        got = out[:nb].cpu().numpy()
        diff = np.flatnonzero(got != np.frombuffer(ref, dtype=np.uint8))
        assert diff.size == 0, (w, case, n, frame, "first differing byte", int(diff[0]))
        back = torch.empty(n, dtype=torch.uint8, device=gpu)
        codec.decode_device_into(out[:nb], codec.parse_header(ref), back, int(s.cuda_stream))
        s.synchronize()
        assert torch.equal(back.cpu(), torch.from_numpy(raw)), (w, case, n, frame)
