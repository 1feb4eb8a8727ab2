"""MI355X tests: HIP kernel numerics vs PyTorch references, and GPU snapshot paths.

Every test here runs the native HIP data plane (``_hsgpu.so``); nothing falls
back to ATen silently -- ``native.require_gpu_lib()`` raises if the library is
missing.
"""

import os

import numpy as np
import pytest
import torch

from hipsnapshot import Snapshot, StateDict
from hipsnapshot.knobs import override_knob, override_slab_size_threshold_bytes
from hipsnapshot import knobs
from hipsnapshot.ops import native
from hipsnapshot.utils.test_utils import assert_state_dict_eq, run_distributed

pytestmark = pytest.mark.gpu

FLOATS = [torch.float32, torch.bfloat16, torch.float16, torch.float64]


def _launch(batch, dev=0):
    batch.launch(dev, int(torch.cuda.current_stream().cuda_stream), sync=True)


def test_pinned_pool_and_dma(gpu):
    n = (64 << 20) + 123
    src = torch.randint(0, 255, (n,), dtype=torch.uint8, device=gpu)
    pb = native.PinnedBuffer(n)
    native.memcpy(0, 0, pb.ptr, src.data_ptr(), n, native.D2H,
                  torch.cuda.current_stream(), sync=True)
    assert torch.equal(pb.as_tensor(n), src.cpu())
    dst = torch.empty_like(src)
    native.memcpy(0, 1, dst.data_ptr(), pb.ptr, n, native.H2D, None, sync=True)
    assert torch.equal(dst, src)
    cached, in_use = native.pinned_stats()
    assert in_use >= n
    pb.release()
    cached_after_release = native.pinned_stats()[0]
    # served from the cache: nothing new registered (which cached block it
    # gets depends on what earlier tests of the process left in the pool)
    pb2 = native.PinnedBuffer(n)
    assert native.pinned_stats()[0] == cached_after_release
    pb2.release()


@pytest.mark.parametrize("dtype", [torch.uint8, torch.bfloat16, torch.float32, torch.int64,
                                   torch.complex64, torch.bool])
def test_gather_contiguous_many_tensors(gpu, dtype):
    torch.manual_seed(0)
    sizes = [1, 7, 64, 1000, 4097, 65536 + 3, 1 << 20, 3]
    ts = [torch.randn(s, device=gpu).to(dtype) if dtype != torch.uint8 else
          torch.randint(0, 255, (s,), dtype=dtype, device=gpu) for s in sizes]
    es = ts[0].element_size()
    total = sum(t.numel() * es for t in ts) + 64 * len(ts)
    out = torch.zeros(total, dtype=torch.uint8, device=gpu)
    b = native.CopyBatch()
    offs, o = [], 3  # deliberately misaligned first offset
    for t in ts:
        offs.append(o)
        b.add(t.data_ptr(), t.dtype, t.stride(), out.data_ptr() + o, t.dtype, [1], [t.numel()], es)
        o += t.numel() * es + 5
    _launch(b)
    for t, off in zip(ts, offs):
        got = out[off: off + t.numel() * es]
        assert torch.equal(got, t.contiguous().view(torch.uint8).view(-1) if dtype != torch.bool
                           else t.view(torch.uint8))


@pytest.mark.parametrize("make", [
    lambda a: a.t(),
    lambda a: a[:, 100:900],
    lambda a: a[::3, 5::7],
    lambda a: a.view(32, 32, 1024).permute(2, 0, 1),
    lambda a: a[7],
    lambda a: a.view(4, 8, 32, 1024)[:, 2:5, ::2, 1:1000].transpose(0, 3),
])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32, torch.int8, torch.float64])
def test_strided_pack_matches_contiguous(gpu, make, dtype):
    a = torch.randn(1024, 1024, device=gpu).to(dtype)
    v = make(a)
    out = torch.empty(v.numel(), dtype=dtype, device=gpu)
    b = native.CopyBatch()
    st = [1] * v.dim()
    for i in range(v.dim() - 2, -1, -1):
        st[i] = st[i + 1] * v.shape[i + 1]
    b.add(v.data_ptr(), dtype, v.stride(), out.data_ptr(), dtype, st, list(v.shape),
          v.element_size())
    _launch(b)
    assert torch.equal(out.view(v.shape), v.contiguous())


@pytest.mark.parametrize("src_dtype", FLOATS, ids=str)
@pytest.mark.parametrize("dst_dtype", FLOATS, ids=str)
def test_scatter_cast_vs_torch(gpu, src_dtype, dst_dtype):
    torch.manual_seed(1)
    src = (torch.randn(257, 129, device=gpu, dtype=torch.float64) * 100).to(src_dtype)
    big = torch.zeros(300, 400, dtype=dst_dtype, device=gpu)
    dst = big[10:267, 50:179]  # strided destination
    b = native.CopyBatch()
    b.add(src.data_ptr(), src_dtype, src.stride(), dst.data_ptr(), dst_dtype, dst.stride(),
          list(src.shape), src.element_size())
    _launch(b)
    ref = src.to(dst_dtype)
    assert torch.equal(dst, ref), (dst - ref).abs().max()
    assert big[:10].abs().sum() == 0 and big[:, :50].abs().sum() == 0


@pytest.mark.parametrize("src_dtype", [torch.float32, torch.bfloat16, torch.float16], ids=str)
@pytest.mark.parametrize("dst_dtype", [torch.float32, torch.bfloat16, torch.float16], ids=str)
@pytest.mark.parametrize("n,off", [(1, 0), (7, 1), (4096 + 5, 0), (3 << 20, 3), ((1 << 22) + 1, 8)])
def test_contiguous_cast_vs_torch(gpu, src_dtype, dst_dtype, n, off):
    """Contiguous casts take the vectorized 8-per-lane path when 16-B aligned
    (off = 0 / 8 elements) and the scalar path otherwise: bit-identical to
    torch's copy_ either way."""
    torch.manual_seed(6)
    src_all = (torch.randn(n + off, device=gpu, dtype=torch.float64) * 300).to(src_dtype)
    src = src_all[off:]
    dst_all = torch.zeros(n + off, dtype=dst_dtype, device=gpu)
    dst = dst_all[off:]
    b = native.CopyBatch()
    b.add(src.data_ptr(), src_dtype, [1], dst.data_ptr(), dst_dtype, [1], [n],
          src.element_size())
    _launch(b)
    ref = src.to(dst_dtype)
    assert torch.equal(dst, ref), (dst.float() - ref.float()).abs().max()
    assert not dst_all[:off].any()


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16, torch.float32])
@pytest.mark.parametrize("n", [1, 127, 128, 1000, 1 << 20, (1 << 20) + 77])
@pytest.mark.parametrize("vpt", [2, 4, 8])
@pytest.mark.parametrize("offset", [0, 1])
def test_fp8_quant_dequant_vs_reference(gpu, dtype, n, vpt, offset):
    """Streaming (hs_fp8_quant_v: aligned source, block within a wave) and
    one-block-per-wave (hs_fp8_quant: misaligned ``offset`` views, f32 blocks
    of 512) quantizers are bit-identical to the torch reference."""
    from hipsnapshot.ops.quant import dequantize_reference, quantize_reference

    torch.manual_seed(2)
    x = (torch.randn(n + offset, device=gpu)
         * torch.logspace(-3, 3, n + offset, device=gpu)).to(dtype)[offset:]
    block = 64 * vpt
    nblocks = (n + block - 1) // block
    q = torch.empty(n, dtype=torch.uint8, device=gpu)
    sc = torch.empty(nblocks, dtype=torch.float32, device=gpu)
    stream = int(torch.cuda.current_stream().cuda_stream)
    native.fp8_quantize(0, x, q, sc, vpt, stream)
    rq, rs = quantize_reference(x, block)
    torch.cuda.synchronize()
    assert torch.equal(sc, rs), (sc - rs).abs().max()
    mism = (q != rq.view(torch.uint8)).sum().item()
    assert mism == 0, f"{mism} fp8 codes differ from torch's float8_e4m3fn cast"
    out = torch.empty(n + offset, dtype=dtype, device=gpu)[offset:]  # misaligned: fallback
    native.fp8_dequantize(0, q, sc, out, vpt, stream)
    ref = dequantize_reference(rq, rs, block, dtype)
    torch.cuda.synchronize()
    assert torch.equal(out, ref)


def _assert_fp8_codes_close(q, rq, min_identical=0.999):
    """e4m3 codes within one fp8 ulp of the reference's, and nearly all equal."""
    a = q.view(torch.float8_e4m3fn).float()
    b = rq.view(torch.float8_e4m3fn).float()
    mag = torch.maximum(a.abs(), b.abs()).clamp_min(2.0 ** -6)
    ulp = torch.exp2(torch.floor(torch.log2(mag)) - 3)
    assert bool(((a - b).abs() <= ulp).all()), (a - b).abs().max()
    same = (q == rq.view(torch.uint8)).float().mean().item()
    assert same >= min_identical, same


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16, torch.float32])
@pytest.mark.parametrize("n", [1, 31, 1000, 1024, 65536 + 77, 3 << 20])
def test_fp8_hadamard_mfma_vs_reference(gpu, dtype, n):
    """MFMA rotation + quantization vs the k-ordered fp32 torch reference.
    fp32 inputs (v_mfma_f32_32x32x2_f32, k-ordered chain): bit-identical.
    bf16 / f16 inputs (v_mfma_f32_32x32x16_{bf16,f16}: the MFMA sums 16
    exact products in its own order): scales within 2 fp32 ulps, every fp8
    code within one fp8 ulp, >= 99.9 % identical, and the round-trip error no
    worse than the reference's.  Dequantization (bf16 MFMA on the widened
    codes, exact row sums)
    is bit-identical to the reference on the kernel's own codes, into every
    float dtype."""
    from hipsnapshot.ops.quant import hadamard_dequantize_reference, hadamard_quantize_reference

    torch.manual_seed(4)
    x = (torch.randn(n, device=gpu) * 3).to(dtype)
    n_pad = (n + 31) // 32 * 32
    nblocks = (n_pad + 127) // 128
    q = torch.zeros(n_pad, dtype=torch.uint8, device=gpu)
    sc = torch.empty(nblocks, dtype=torch.float32, device=gpu)
    stream = int(torch.cuda.current_stream().cuda_stream)
    native.fp8_hadamard_quantize(0, x, q, sc, stream)
    rq, rs = hadamard_quantize_reference(x, 128)
    torch.cuda.synchronize()
    if dtype == torch.float32:
        assert torch.equal(sc, rs), (sc - rs).abs().max()
        assert torch.equal(q, rq.view(torch.uint8)), (q != rq.view(torch.uint8)).sum()
    else:
        assert torch.allclose(sc, rs, rtol=2.0 ** -22, atol=0), ((sc - rs) / rs).abs().max()
        _assert_fp8_codes_close(q, rq)
    for out_dtype in (dtype, torch.float64):
        out = torch.empty(n, dtype=out_dtype, device=gpu)
        native.fp8_hadamard_dequantize(0, q, sc, out, stream)
        ref = hadamard_dequantize_reference(q.view(torch.float8_e4m3fn), sc, n, out_dtype)
        torch.cuda.synchronize()
        assert torch.equal(out, ref), (out_dtype, (out.float() - ref.float()).abs().max())
    out = out.to(dtype)
    if dtype != torch.float32 and n >= 1000:
        rt_ref = hadamard_dequantize_reference(rq, rs, n, torch.float32)
        err_gpu = (out.float() - x.float()).norm()
        err_ref = (rt_ref - x.float()).norm()
        assert err_gpu <= err_ref * 1.01, (err_gpu, err_ref)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16, torch.float32])
@pytest.mark.parametrize("n", [1, 31, 32, 1000, 2048, 4096 + 17, (1 << 20) + 5, 3 << 20])
def test_mx8_quant_dequant_vs_reference(gpu, dtype, n):
    """MX fp8 (E8M0 scale per 32, hs_mx8_quant/dequant): payload, padding and
    scale bytes bit-identical to the torch reference; dequantization into
    every float dtype bit-identical too."""
    from hipsnapshot.ops.quant import mx_dequantize_reference, mx_quantize_reference

    torch.manual_seed(5)
    x = (torch.randn(n, device=gpu) * torch.logspace(-12, 12, n, device=gpu)).to(dtype)
    if n >= 1000:  # special values: zero block, inf, nan
        x[:32] = 0
        x[40] = float("inf")
        x[77] = float("nan")
    payload = (n + 15) // 16 * 16
    nb = (n + 31) // 32
    blob = torch.full((payload + nb,), 0xAB, dtype=torch.uint8, device=gpu)  # no zero-fill
    stream = int(torch.cuda.current_stream().cuda_stream)
    native.mx8_quantize(0, x, blob[:payload], blob[payload:], stream)
    rq, rs = mx_quantize_reference(x)
    torch.cuda.synchronize()
    assert torch.equal(blob[payload:], rs), (blob[payload:] != rs).sum()
    assert torch.equal(blob[:n], rq.view(torch.uint8)), (blob[:n] != rq.view(torch.uint8)).sum()
    assert not blob[n:payload].any()  # padding written as zeros
    for out_dtype in (torch.bfloat16, torch.float16, torch.float32, torch.float64):
        out = torch.empty(n, dtype=out_dtype, device=gpu)
        native.mx8_dequantize(0, blob[:n], blob[payload:], out, stream)
        ref = mx_dequantize_reference(rq, rs, out_dtype)
        torch.cuda.synchronize()
        assert torch.equal(out.isnan(), ref.isnan())
        ok = ~ref.isnan()
        assert torch.equal(out[ok], ref[ok]), (out_dtype, (out[ok] != ref[ok]).sum())


def test_mx8_snapshot_gpu(gpu, tmp_path):
    """Default fp8 quantized save is the MX layout; GPU save + GPU restore
    equal the torch reference, and a CPU restore of the same blob too."""
    from hipsnapshot.ops.quant import mx_dequantize_reference, mx_quantize_reference

    w = torch.randn(777, 333, device=gpu, dtype=torch.bfloat16)
    Snapshot.take(str(tmp_path / "s"), {"sd": StateDict(w=w)}, quantize=["sd/*"])
    e = Snapshot(str(tmp_path / "s")).get_manifest()["0/sd/w"]
    assert e.quant["format"] == "fp8_e4m3fn_mx"
    q, s = mx_quantize_reference(w)
    ref = mx_dequantize_reference(q, s, torch.bfloat16).view(w.shape)
    out = torch.zeros_like(w)
    Snapshot(str(tmp_path / "s")).restore({"sd": StateDict(w=out)})
    assert torch.equal(out, ref)
    host = torch.zeros(w.shape, dtype=torch.bfloat16)
    Snapshot(str(tmp_path / "s")).restore({"sd": StateDict(w=host)})
    assert torch.equal(host, ref.cpu())


def test_fp8_hadamard_snapshot_gpu(gpu, tmp_path):
    from hipsnapshot.ops.quant import hadamard_dequantize_reference, hadamard_quantize_reference
    from hipsnapshot.utils.test_utils import env

    w = torch.randn(777, 333, device=gpu, dtype=torch.bfloat16)
    with env(HIPSNAPSHOT_FP8_FORMAT="hadamard32"):
        Snapshot.take(str(tmp_path / "s"), {"sd": StateDict(w=w)}, quantize=["sd/*"])
    out = torch.zeros_like(w)
    Snapshot(str(tmp_path / "s")).restore({"sd": StateDict(w=out)})
    # the blob holds the kernel's codes (bf16 MFMA): the restore is their
    # exact dequantization, and they match the fp32 reference within an ulp
    n_pad = (w.numel() + 31) // 32 * 32
    q = torch.zeros(n_pad, dtype=torch.uint8, device=gpu)
    s = torch.empty((n_pad + 127) // 128, dtype=torch.float32, device=gpu)
    native.fp8_hadamard_quantize(0, w, q, s, int(torch.cuda.current_stream().cuda_stream))
    ref = hadamard_dequantize_reference(q.view(torch.float8_e4m3fn), s, w.numel(),
                                        torch.bfloat16).view(w.shape)
    assert torch.equal(out, ref)
    rq, _rs = hadamard_quantize_reference(w, 128)
    _assert_fp8_codes_close(q, rq)


def test_gpu_snapshot_roundtrip(gpu, tmp_path):
    torch.manual_seed(3)
    a = torch.randn(512, 256, device=gpu)
    sd = StateDict(
        w=torch.randn(1000, 300, device=gpu, dtype=torch.bfloat16),
        t=a.t(),                                   # strided view
        col=a[:, 10:100],                          # column shard-like view
        small=[torch.randn(i + 1, device=gpu) for i in range(50)],  # slab members
        i64=torch.arange(1000, device=gpu),
        cpu=torch.randn(77),
        step=3,
    )
    ref = {k: (v.clone() if isinstance(v, torch.Tensor) else
               [x.clone() for x in v] if isinstance(v, list) else v) for k, v in sd.items()}
    with override_slab_size_threshold_bytes(1 << 20):
        Snapshot.take(str(tmp_path / "s"), {"sd": sd})
    out = StateDict(
        w=torch.zeros(1000, 300, device=gpu, dtype=torch.bfloat16),
        t=torch.zeros(256, 512, device=gpu),
        col=torch.zeros(1024, 180, device=gpu)[::2, ::2],   # strided destination
        small=[torch.zeros(i + 1, device=gpu) for i in range(50)],
        i64=torch.zeros(1000, dtype=torch.int64, device=gpu),
        cpu=torch.zeros(77),
    )
    Snapshot(str(tmp_path / "s")).restore({"sd": out})
    torch.cuda.synchronize()
    assert_state_dict_eq({k: out[k] for k in ref}, ref)


def test_gpu_restore_with_dtype_cast(gpu, tmp_path):
    w = torch.randn(300, 200, device=gpu)
    Snapshot.take(str(tmp_path / "s"), {"sd": StateDict(w=w)})
    out = torch.zeros(300, 200, device=gpu, dtype=torch.bfloat16)
    Snapshot(str(tmp_path / "s")).read_object("0/sd/w", obj_out=out)
    # dtype differs -> not in place; result returned on host, cast on copy
    got = Snapshot(str(tmp_path / "s")).read_object("0/sd/w")
    assert torch.equal(got, w.cpu())


def test_async_take_hbm_freeze_is_consistent(gpu, tmp_path):
    w = torch.randn(4096, 1024, device=gpu)
    small = torch.randn(100, device=gpu)
    ref_w, ref_s = w.clone(), small.clone()
    pending = Snapshot.async_take(str(tmp_path / "s"), {"sd": StateDict(w=w, s=small)})
    w.add_(1.0)        # enqueued after the freeze on the same stream
    small.mul_(0)
    pending.wait()
    out = StateDict(w=torch.zeros_like(w), s=torch.zeros_like(small))
    Snapshot(str(tmp_path / "s")).restore({"sd": out})
    assert torch.equal(out["w"], ref_w) and torch.equal(out["s"], ref_s)


def test_async_take_host_fallback_when_hbm_short(gpu, tmp_path):
    w = torch.randn(1024, 1024, device=gpu)
    ref = w.clone()
    with override_knob("HBM_STAGING_RESERVE_BYTES", str(1 << 50)):
        pending = Snapshot.async_take(str(tmp_path / "s"), {"sd": StateDict(w=w)})
    w.zero_()
    pending.wait()
    assert torch.equal(Snapshot(str(tmp_path / "s")).read_object("0/sd/w"), ref.cpu())


@pytest.mark.parametrize("compression", ["none", "hsz1"])
def test_async_take_unfrozen_large_tensor_not_raced(gpu, tmp_path, compression):
    """No HBM room: a 256 MiB contiguous tensor (above the slab threshold) is
    copied straight from the LIVE tensor by the asynchronous SDMA path, with
    its on-device hash.  async_take must not return before that copy and hash
    are done: a zero_() right after it must not reach the snapshot."""
    w = torch.randn(64 << 20, device=gpu)
    ref = w.clone()
    with override_knob("HBM_STAGING_RESERVE_BYTES", str(1 << 50)), \
            override_knob("CHECKSUM", "1"):
        pending = Snapshot.async_take(str(tmp_path / "s"), {"sd": StateDict(w=w)},
                                      compression=compression)
        w.zero_()
        pending.wait()
    got = torch.zeros_like(w)
    Snapshot(str(tmp_path / "s")).restore({"sd": StateDict(w=got)})
    assert torch.equal(got, ref)
    from hipsnapshot.verify import verify_snapshot

    assert verify_snapshot(str(tmp_path / "s")).ok


def test_async_take_partial_hbm_freeze(gpu, tmp_path):
    """Arena smaller than the state: the requests that fit are frozen in HBM,
    the rest is host-staged before async_take returns -- both consistent."""
    from hipsnapshot.io.batcher import GPUBatchedBufferStager
    from hipsnapshot.engine import hbm_staging

    big = torch.randn(2048, 1024, device=gpu)            # 8 MiB: its own blob
    small = [torch.randn(1000 + i, device=gpu) for i in range(8)]  # one slab
    refs = [big.clone()] + [t.clone() for t in small]
    seen = {}
    orig = hbm_staging.freeze_device_state

    def spy(write_reqs, plan=None, **kw):
        out = orig(write_reqs, plan, **kw)
        seen["frozen"] = out
        seen["kinds"] = [(type(wr.buffer_stager).__name__, hbm_staging.is_deferrable(wr))
                         for wr in write_reqs]
        return out

    with override_knob("HBM_STAGING_MAX_BYTES", str(1 << 20)), \
            override_slab_size_threshold_bytes(4 << 20):
        hbm_staging.freeze_device_state = spy
        try:
            pending = Snapshot.async_take(str(tmp_path / "s"),
                                          {"sd": StateDict(big=big, small=small)})
        finally:
            hbm_staging.freeze_device_state = orig
    big.add_(1.0)
    for t in small:
        t.mul_(0)
    pending.wait()
    assert 0 < seen["frozen"][0] <= 1 << 20
    assert (GPUBatchedBufferStager.__name__, True) in seen["kinds"]   # slab frozen
    assert ("TensorBufferStager", False) in seen["kinds"]             # big: host path
    out = StateDict(big=torch.zeros_like(big), small=[torch.zeros_like(t) for t in small])
    Snapshot(str(tmp_path / "s")).restore({"sd": out})
    assert torch.equal(out["big"], refs[0])
    for got, ref in zip(out["small"], refs[1:]):
        assert torch.equal(got, ref)


def test_fp8_quantized_save_gpu(gpu, tmp_path):
    from hipsnapshot.ops.quant import dequantize_reference, quantize_reference

    from hipsnapshot.utils.test_utils import env

    w = torch.randn(1000, 333, device=gpu, dtype=torch.bfloat16)
    with env(HIPSNAPSHOT_FP8_FORMAT="block"):  # the fp32-scale layout (MX: test_mx8_*)
        Snapshot.take(str(tmp_path / "s"), {"sd": StateDict(w=w)}, quantize=["sd/*"])
    out = torch.zeros_like(w)
    Snapshot(str(tmp_path / "s")).restore({"sd": StateDict(w=out)})
    q, s = quantize_reference(w, 128)
    ref = dequantize_reference(q, s, 128, torch.bfloat16).view(w.shape)
    assert torch.equal(out, ref)
    size = sum(os.path.getsize(os.path.join(r, f)) for r, _, fs in os.walk(tmp_path / "s")
               for f in fs if not f.startswith("."))
    assert size < w.numel() * 2 * 0.55  # ~half of the bf16 bytes


def test_uvm_managed_tensor(gpu, tmp_path):
    from hipsnapshot.ops.uvm import is_uvm_tensor, new_managed_tensor

    t = new_managed_tensor([256, 64], torch.float32, 0)
    t.copy_(torch.randn(256, 64, device=gpu))
    assert is_uvm_tensor(t) and not is_uvm_tensor(torch.zeros(3, device=gpu))
    Snapshot.take(str(tmp_path / "s"), {"sd": StateDict(t=t)})
    out = new_managed_tensor([256, 64], torch.float32, 0)
    out.zero_()
    Snapshot(str(tmp_path / "s")).restore({"sd": StateDict(t=out)})
    torch.cuda.synchronize()
    assert torch.equal(out, t)


@pytest.mark.parametrize("where", ["host", "device", None])
def test_uvm_placed_save_restore(gpu, tmp_path, where, monkeypatch):
    """Managed tables placed in host DRAM are written in place by a blocking
    take (no DMA, no pinned copy), copied by an async take (it must not alias
    live memory), and both restore bitwise with verified checksums; tables
    placed in HBM keep the DMA path.  The take waits for kernels still
    writing the table."""
    from hipsnapshot.engine import staging
    from hipsnapshot.ops.uvm import new_managed_tensor, place, residency
    from hipsnapshot.verify import verify_snapshot

    from hipsnapshot import knobs

    t = new_managed_tensor([4096, 1024], torch.float32, 0)
    if where is not None:
        place(t, where)
    torch.cuda.synchronize()
    # never-placed pages are in host DRAM unless XNACK migrates them
    host = where == "host" or (where is None and knobs.uvm_assume_host())
    assert residency(t) == ("host" if host else where or "unknown")
    views = []
    real = staging.managed_host_view
    monkeypatch.setattr(staging, "managed_host_view",
                        lambda x, p: views.append(x.numel()) or real(x, p))
    with override_slab_size_threshold_bytes(1 << 20):  # t is its own blob
        t.normal_()
        ref = t.clone()
        Snapshot.take(str(tmp_path / "s"), {"sd": StateDict(t=t)})  # normal_ may still run
        assert views == ([t.numel()] if host else [])
        pending = Snapshot.async_take(str(tmp_path / "a"), {"sd": StateDict(t=t)})
        t.add_(1.0)  # after the async take's capture
        pending.wait()
    assert len(views) == (1 if host else 0)
    out_m = new_managed_tensor([4096, 1024], torch.float32, 0)
    if where is not None:
        place(out_m, where)
    for p in ("s", "a"):
        assert verify_snapshot(str(tmp_path / p)).ok
        out = torch.zeros_like(ref)
        Snapshot(str(tmp_path / p)).restore({"sd": StateDict(t=out)})
        assert torch.equal(out, ref), p
        # into placed UVM pages: host DRAM ones are read into in place
        out_m.zero_()
        n = len(views)
        Snapshot(str(tmp_path / p)).restore({"sd": StateDict(t=out_m)})
        torch.cuda.synchronize()
        assert torch.equal(out_m, ref), p
        assert len(views) == n + (1 if host else 0)


def _fsdp_gpu_worker(path):
    import torch.distributed as dist
    from torch.distributed.device_mesh import init_device_mesh

    from hipsnapshot.models.llama import LlamaConfig, build_fsdp_llama

    mesh = init_device_mesh("cuda", (dist.get_world_size(),))
    m = build_fsdp_llama(LlamaConfig.tiny(), torch.device("cuda", 0), torch.bfloat16, mesh=mesh)
    ref = {k: v.full_tensor().clone() for k, v in m.state_dict().items()}
    Snapshot.take(path, {"model": m})
    pending = Snapshot.async_take(path + "_a", {"model": m})
    pending.wait()
    for p in m.parameters():
        p._local_tensor.zero_()
    Snapshot(path + "_a").restore({"model": m})
    torch.cuda.synchronize()
    for k, v in m.state_dict().items():
        assert torch.equal(v.full_tensor(), ref[k]), k


def test_fsdp2_rccl_single_rank(gpu, tmp_path):
    run_distributed(_fsdp_gpu_worker, 1, str(tmp_path / "f"), backend="nccl")


def _fsdp_gpu_optim_worker(path):
    """FSDP2 + AdamW in HBM: an async take after training steps, restored
    into a fresh model and a fresh AdamW (no state tensors yet: created by a
    zero step, then filled by the native restore job)."""
    import torch.distributed as dist
    from torch.distributed.device_mesh import init_device_mesh

    from hipsnapshot.models.llama import LlamaConfig, build_fsdp_llama

    mesh = init_device_mesh("cuda", (dist.get_world_size(),))

    def build(seed):
        torch.manual_seed(seed)
        m = build_fsdp_llama(LlamaConfig.tiny(), torch.device("cuda", 0), torch.float32,
                             mesh=mesh)
        return m, torch.optim.AdamW(m.parameters(), lr=1e-3, weight_decay=0.1)

    m, opt = build(0)
    for _ in range(2):
        m(torch.randint(0, 256, (2, 16), device="cuda")).float().logsumexp(-1).mean().backward()
        opt.step()
        opt.zero_grad()
    ref_m = {k: v.full_tensor().clone() for k, v in m.state_dict().items()}
    ref_o = {(i, n): (v.full_tensor() if hasattr(v, "full_tensor") else v).clone()
             for i, st in opt.state_dict()["state"].items() for n, v in st.items()}
    Snapshot.async_take(path, {"model": m, "optim": opt}).wait()
    m2, opt2 = build(1)
    Snapshot(path).restore({"model": m2, "optim": opt2}, verify=True)
    torch.cuda.synchronize()
    for k, v in m2.state_dict().items():
        assert torch.equal(v.full_tensor(), ref_m[k]), k
    got = {(i, n): (v.full_tensor() if hasattr(v, "full_tensor") else v)
           for i, st in opt2.state_dict()["state"].items() for n, v in st.items()}
    assert set(got) == set(ref_o)
    for k, v in got.items():
        assert torch.equal(v.cpu(), ref_o[k].cpu()), k


def test_fsdp2_adamw_restores_into_fresh_optimizer(gpu, tmp_path):
    run_distributed(_fsdp_gpu_optim_worker, 1, str(tmp_path / "o"), backend="nccl")


def test_rccl_forced_collectives_match_gloo(gpu, tmp_path, monkeypatch):
    """HIPSNAPSHOT_FORCE_COLLECTIVES: a one-rank RCCL group runs every
    collective the planner and commit use -- framed all_gather_into_tensor
    with its overflow round, broadcast with a device, barrier(device_ids),
    scatter, the store bootstrap broadcast, the helper thread's manifest
    gather, a self batch_isend_irecv -- around a whole FSDP2 take /
    async_take / restore, with results identical to the gloo run of the
    same worker.  The RCCL debug log must show the collectives ran."""
    import json
    import shutil

    import dist_workers as W

    logdir = tmp_path / "rccl"
    logdir.mkdir()
    monkeypatch.setenv("NCCL_DEBUG", "INFO")
    monkeypatch.setenv("NCCL_DEBUG_SUBSYS", "INIT,COLL,P2P")
    monkeypatch.setenv("NCCL_DEBUG_FILE", str(logdir / "rccl.%p.log"))
    run_distributed(W.forced_collectives, 1, str(tmp_path / "n"), str(tmp_path / "n.json"),
                    True, backend="nccl")
    monkeypatch.delenv("NCCL_DEBUG")
    run_distributed(W.forced_collectives, 1, str(tmp_path / "g"), str(tmp_path / "g.json"),
                    True, backend="gloo")
    rn = json.loads((tmp_path / "n.json").read_text())
    rg = json.loads((tmp_path / "g.json").read_text())
    assert rn.pop("backend") == "nccl" and rg.pop("backend") == "gloo"
    assert rn == rg
    log = "".join(f.read_text(errors="replace") for f in logdir.iterdir())
    ops = {op: log.count(f"{op}: opCount") for op in ("AllGather", "Broadcast", "AllReduce")}
    assert all(n > 0 for n in ops.values()), ops
    art = os.environ.get("HSTEST_ARTIFACTS")
    if art:  # the GPU runs keep the RCCL log (profiles/r5/rccl_forced/)
        os.makedirs(art, exist_ok=True)
        for f in logdir.iterdir():
            shutil.copy(f, os.path.join(art, f.name))
        with open(os.path.join(art, "rccl_forced_ops.json"), "w") as f:
            json.dump(ops, f)


def _multirank_gpu_worker(path, phase, compression=None):
    """Several ranks sharing cuda:0 with gloo metadata collectives: exercises
    the multi-rank take/restore logic (partitioning, manifest merge, sharded
    resharding, HBM freeze, store-barrier commit) on device tensors."""
    import torch.distributed as dist
    from torch.distributed.device_mesh import init_device_mesh
    from torch.distributed.tensor import DTensor, Shard

    rank, ws = dist.get_rank(), dist.get_world_size()
    torch.manual_seed(0)
    full = torch.randn(96, 2048, device="cuda:0")
    mesh = init_device_mesh("cuda", (ws,))
    rows = 96 // ws
    local = full[rank * rows:(rank + 1) * rows].clone()
    dt = DTensor.from_local(local, mesh, [Shard(0)], run_check=False)
    rep = torch.arange(1000, device="cuda:0", dtype=torch.float32)
    if phase == "save":
        Snapshot.take(path, {"m": StateDict(w=dt, rep=rep, mine=torch.full((5,), float(rank),
                                                                            device="cuda:0"))},
                      replicated=["m/rep"], compression=compression)
        p = Snapshot.async_take(path + "_a", {"m": StateDict(w=dt, rep=rep)},
                                replicated=["m/rep"], compression=compression)
        local.add_(1)  # after the freeze: must not leak
        p.wait()
        local.sub_(1)
    else:
        out = torch.zeros_like(local)
        odt = DTensor.from_local(out, mesh, [Shard(0)], run_check=False)
        r2 = torch.zeros_like(rep)
        Snapshot(path + "_a").restore({"m": StateDict(w=odt, rep=r2)})
        torch.cuda.synchronize()
        assert torch.equal(out, full[rank * rows:(rank + 1) * rows]), rank
        assert torch.equal(r2, rep)
        whole = torch.zeros(96, 2048, device="cuda:0")
        Snapshot(path).read_object("0/m/w", obj_out=whole)
        assert torch.equal(whole, full)


@pytest.mark.parametrize("save_ws,load_ws", [(2, 2), (2, 3), (4, 2)])
def test_multirank_gpu_tensors_gloo(gpu, tmp_path, save_ws, load_ws):
    p = str(tmp_path / "mr")
    run_distributed(_multirank_gpu_worker, save_ws, p, "save", backend="gloo")
    run_distributed(_multirank_gpu_worker, load_ws, p, "load", backend="gloo")


# ---- HSZ1 lossless codec kernels ------------------------------------------------

def _codec_inputs():
    g = torch.Generator().manual_seed(7)
    w_bf16 = (torch.randn(3_000_001, generator=g) * 0.02).to(torch.bfloat16)
    rnd = torch.randint(0, 256, (200_003,), dtype=torch.uint8, generator=g)
    # escapes in every frame: 14 common high bytes + a sprinkle of rare ones
    hi = torch.randint(60, 74, (400_000,), dtype=torch.uint8, generator=g)
    hi[::997] = torch.randint(0, 256, (hi[::997].numel(),), dtype=torch.uint8, generator=g)
    esc = torch.stack([torch.randint(0, 256, (400_000,), dtype=torch.uint8, generator=g), hi],
                      1).reshape(-1)
    return {"bf16": w_bf16.view(torch.uint8), "random": rnd, "escapes": esc,
            "fp32": (torch.randn(500_000, generator=g) * 1e-3).view(torch.uint8)}


@pytest.mark.parametrize("w", [1, 2, 4, 8])
@pytest.mark.parametrize("kind", ["bf16", "random", "escapes", "fp32"])
@pytest.mark.parametrize("grid_cap", [0, 3])
def test_hsz_encode_gpu_bit_exact_vs_reference(gpu, w, kind, grid_cap, monkeypatch):
    """``grid_cap`` 3: each workgroup walks several frames (async-take drains
    cap the encoder's grid) -- same bytes."""
    from hipsnapshot.ops import codec

    prev = native.set_thread_grid_cap(grid_cap)
    try:
        _hsz_encode_bit_exact(gpu, w, kind)
    finally:
        native.set_thread_grid_cap(prev)


def _hsz_encode_bit_exact(gpu, w, kind):
    from hipsnapshot.ops import codec

    host = _codec_inputs()[kind]
    # 2 * 65536 + 32003: the last frame holds 8000 fp32 elements and a 3-byte
    # tail (a mode-2 frame with a tail when w == 4)
    for n in (host.numel(), host.numel() - 7, 4096 * 16 + 3, 2 * 65536 + 32003):
        h = host[:n].contiguous()
        ref = codec.encode_reference(h.numpy().tobytes(), w, 64 * 1024)
        d = h.to(gpu)
        s = torch.cuda.current_stream()
        out, total, _ = codec.encode_device(d, w, int(s.cuda_stream), 64 * 1024)
        s.synchronize()
        nb = int(total.item())
        assert nb == len(ref), (kind, w, n)
        got = out[:nb].cpu().numpy()
        diff = np.flatnonzero(got != np.frombuffer(ref, dtype=np.uint8))
        assert diff.size == 0, (kind, w, n, "first differing byte", int(diff[0]))
        # GPU decode of the whole blob and of a middle frame range
        hdr = codec.parse_header(ref)
        back = torch.empty(n, dtype=torch.uint8, device=gpu)
        codec.decode_device_into(out[:nb], hdr, back, int(s.cuda_stream))
        assert torch.equal(back.cpu(), h), (kind, w, n)
        if hdr.n_frames >= 3:
            lo, _ = hdr.frame_range(1)
            _, hi_ = hdr.frame_range(2)
            part = torch.empty(hi_ - lo, dtype=torch.uint8, device=gpu)
            base = hdr.offsets[1]
            codec.decode_device_into(out[base:nb], hdr, part, int(s.cuda_stream), first=1,
                                     count=2, blob_base=base)
            assert torch.equal(part.cpu(), h[lo:hi_])


def test_hsz_gpu_length_limited_huffman_frame(gpu):
    # the GPU's wave-parallel Huffman construction must apply the same
    # length limit (Kraft fix-up) as the reference, byte for byte
    from hipsnapshot.ops import codec
    from hipsnapshot.utils.test_utils import hsz_deep_tree_frame

    raw = hsz_deep_tree_frame()
    ref = codec.encode_reference(raw, 2, frame_bytes=len(raw))
    d = torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(gpu)
    s = torch.cuda.current_stream()
    out, total, _ = codec.encode_device(d, 2, int(s.cuda_stream), len(raw))
    s.synchronize()
    nb = int(total.item())
    assert nb == len(ref)
    got = out[:nb].cpu().numpy()
    diff = np.flatnonzero(got != np.frombuffer(ref, dtype=np.uint8))
    assert diff.size == 0, ("first differing byte", int(diff[0]))
    back = torch.empty_like(d)
    codec.decode_device_into(out[:nb], codec.parse_header(ref), back, int(s.cuda_stream))
    assert torch.equal(back, d)


def test_hsz_gpu_large_blob_ratio(gpu):
    from hipsnapshot.ops import codec

    x = (torch.randn(64 << 20, device=gpu) / 64).to(torch.bfloat16)  # 128 MiB
    s = torch.cuda.current_stream()
    out, total, _ = codec.encode_device(x.view(torch.uint8), 2, int(s.cuda_stream))
    s.synchronize()
    nb = int(total.item())
    assert 0.66 < nb / (x.numel() * 2) < 0.68  # mode-2 (Huffman) frames
    nf = codec.n_frames_for(x.numel() * 2, codec.DEFAULT_FRAME_BYTES)
    hdr = codec.parse_header(out[:codec.payload_start(nf)].cpu().numpy().tobytes())
    back = torch.empty_like(x)
    codec.decode_device_into(out[:nb], hdr, back.view(torch.uint8), int(s.cuda_stream))
    assert torch.equal(back.view(torch.int16), x.view(torch.int16))


def test_hsz_gpu_fp32_blob_ratio(gpu):
    from hipsnapshot.ops import codec

    x = torch.randn(32 << 20, device=gpu) / 64  # 128 MiB fp32
    s = torch.cuda.current_stream()
    out, total, _ = codec.encode_device(x.view(torch.uint8), 4, int(s.cuda_stream))
    s.synchronize()
    nb = int(total.item())
    assert 0.83 < nb / (x.numel() * 4) < 0.845  # mode-2 frames (mode 1 would be 0.876)
    nf = codec.n_frames_for(x.numel() * 4, codec.DEFAULT_FRAME_BYTES)
    hdr = codec.parse_header(out[:codec.payload_start(nf)].cpu().numpy().tobytes())
    back = torch.empty_like(x)
    codec.decode_device_into(out[:nb], hdr, back.view(torch.uint8), int(s.cuda_stream))
    assert torch.equal(back.view(torch.int32), x.view(torch.int32))


def _corruptions(blob: bytes, w: int):
    """(name, corrupted blob) pairs that the host decoder rejects."""
    from hipsnapshot.ops import codec

    h = codec.parse_header(blob)
    f1 = h.offsets[1]
    n = h.frame_bytes // w
    lane_tab = f1 + 32 + (w - 1) * n   # mode-2 body: low bytes, then the lane table

    def patch(off, val):
        b = bytearray(blob)
        b[off:off + len(val)] = val
        return bytes(b)

    out = [("mode byte", patch(f1, b"\x09")),
           ("code length > max", patch(f1 + 24, b"\xff")),
           ("lane table overflow", patch(lane_tab, b"\xff\xff"))]
    if codec.frame_modes(blob)[1] == 2:
        # every lane claims 0 stream bytes: lanes read past their own streams
        out.append(("lane overrun", patch(lane_tab, bytes(2 * 256))))
    return out


@pytest.mark.parametrize("w", [2, 4])
def test_hsz_gpu_decode_rejects_corrupt_frames(gpu, w):
    """Every frame the host decoder rejects (-74) makes the GPU decode raise
    too, instead of leaving the output unwritten."""
    from hipsnapshot.ops import codec

    g = torch.Generator().manual_seed(3)
    x = (torch.randn(3 * 65536 // w, generator=g) * 0.02)
    x = x.to(torch.bfloat16) if w == 2 else x
    raw = x.view(torch.uint8).numpy().tobytes()
    blob = codec.encode_reference(raw, w, 64 * 1024)
    assert codec.frame_modes(blob)[1] == 2
    s = torch.cuda.current_stream()
    for name, bad in _corruptions(blob, w):
        with pytest.raises(Exception):
            codec.decode_cpu(bad)
        d = torch.frombuffer(bytearray(bad), dtype=torch.uint8).to(gpu)
        out = torch.empty(len(raw), dtype=torch.uint8, device=gpu)
        with pytest.raises(ValueError, match="corrupt HSZ1"):
            codec.decode_device_into(d, codec.parse_header(bad), out, int(s.cuda_stream))
    # the intact blob still decodes (no sticky error state)
    d = torch.frombuffer(bytearray(blob), dtype=torch.uint8).to(gpu)
    out = torch.empty(len(raw), dtype=torch.uint8, device=gpu)
    codec.decode_device_into(d, codec.parse_header(blob), out, int(s.cuda_stream))
    assert out.cpu().numpy().tobytes() == raw


@pytest.mark.parametrize("w", [2, 4])
def test_hsz_gpu_decode_bit_exact(gpu, w):
    """The mode-2 decoder reproduces the input bit for bit: escapes (values
    outside the 15-entry dictionary), a short last frame with tail bytes, and
    an output that is not 16-B aligned (byte-store path)."""
    from hipsnapshot.ops import codec
    g = torch.Generator().manual_seed(11)
    n = (5 * 65536 + 4 * 1000 + 8) // w
    x = torch.randn(n, generator=g) * 0.02
    x[::97] *= 1e-6   # tiny exponents: escapes
    x[::1013] *= 1e4  # large exponents: escapes
    x = x.to(torch.bfloat16) if w == 2 else x
    raw = x.view(torch.uint8).numpy().tobytes() + b"\x01\x02\x03"[: (w - 1)]
    blob = codec.encode_reference(raw, w, 64 * 1024)
    assert 2 in codec.frame_modes(blob)
    hdr = codec.parse_header(blob)
    s = torch.cuda.current_stream()
    d = torch.frombuffer(bytearray(blob), dtype=torch.uint8).to(gpu)
    for shift in (0, 1):
        buf = torch.full((len(raw) + shift,), 0xAB, dtype=torch.uint8, device=gpu)
        out = buf[shift:]
        codec.decode_device_into(d, hdr, out, int(s.cuda_stream))
        assert out.cpu().numpy().tobytes() == raw, (variant, shift)


@pytest.mark.parametrize("direct", [True, False])
def test_gpu_restore_of_corrupt_compressed_blob_raises(gpu, tmp_path, direct):
    from hipsnapshot.knobs import override_is_batching_disabled
    from hipsnapshot.ops import codec

    big = (torch.randn(3000, 1024, device=gpu) * 0.02).to(torch.bfloat16)
    path = str(tmp_path / "c")
    with override_is_batching_disabled(True):
        Snapshot.take(path, {"sd": StateDict(big=big)}, compression="hsz1")
    f = os.path.join(path, "0", "sd", "big")
    blob = open(f, "rb").read()
    h = codec.parse_header(blob)
    with open(f, "r+b") as fh:  # frame 2's mode byte
        fh.seek(h.offsets[2])
        fh.write(b"\x09")
    # direct: decoded straight into the target; else via scratch + cast copy
    out = StateDict(big=torch.zeros(3000, 1024, device=gpu,
                                    dtype=torch.bfloat16 if direct else torch.float32))
    with override_is_batching_disabled(True), pytest.raises(Exception, match="corrupt HSZ1"):
        Snapshot(path).restore({"sd": out})
    torch.cuda.synchronize()


# ---- HSZ1 compressed snapshots on the GPU path ---------------------------------

def _compressible_state(gpu):
    torch.manual_seed(11)
    a = torch.randn(512, 256, device=gpu)
    return StateDict(
        w=(torch.randn(1000, 300, device=gpu) * 0.02).to(torch.bfloat16),
        big=(torch.randn(3000, 1024, device=gpu) * 0.02).to(torch.bfloat16),
        t=a.t(),                                   # strided view, fp32
        col=a[:, 10:100],
        small=[torch.randn(i + 1000, device=gpu) for i in range(20)],  # slab members
        h=torch.randn(70_001, device=gpu, dtype=torch.float16),
        i64=torch.arange(100_000, device=gpu),
        cpu=torch.randn(77),
        step=3,
    )


def _clone_state(sd):
    return {k: (v.clone() if isinstance(v, torch.Tensor) else
                [x.clone() for x in v] if isinstance(v, list) else v) for k, v in sd.items()}


@pytest.mark.parametrize("slab", [1 << 20, 64 << 20])
def test_gpu_compressed_snapshot_roundtrip(gpu, tmp_path, slab):
    sd = _compressible_state(gpu)
    ref = _clone_state(sd)
    with override_slab_size_threshold_bytes(slab):
        snap = Snapshot.take(str(tmp_path / "s"), {"sd": sd}, compression="hsz1")
    man = snap.get_manifest()
    assert man["0/sd/big"].codec is not None and man["0/sd/cpu"].codec is None
    total = sum(os.path.getsize(os.path.join(r, f)) for r, _, fs in os.walk(tmp_path / "s")
                for f in fs)
    raw = sum(v.numel() * v.element_size() for v in ref.values() if isinstance(v, torch.Tensor))
    assert total < raw  # the bf16 payload shrank
    out = StateDict(
        w=torch.zeros(1000, 300, device=gpu, dtype=torch.bfloat16),
        big=torch.zeros(3000, 1024, device=gpu, dtype=torch.bfloat16),
        t=torch.zeros(256, 512, device=gpu),
        col=torch.zeros(1024, 180, device=gpu)[::2, ::2],   # strided destination
        small=[torch.zeros(i + 1000, device=gpu) for i in range(20)],
        h=torch.zeros(70_001, device=gpu, dtype=torch.float16),
        i64=torch.zeros(100_000, dtype=torch.int64, device=gpu),
        cpu=torch.zeros(77),
    )
    Snapshot(str(tmp_path / "s")).restore({"sd": out})
    torch.cuda.synchronize()
    assert_state_dict_eq({k: out[k] for k in ref}, ref)
    # host read of a compressed device blob (CPU decoder)
    got = Snapshot(str(tmp_path / "s")).read_object("0/sd/big")
    assert torch.equal(got, ref["big"].cpu())


def test_gpu_compressed_async_take(gpu, tmp_path):
    w = (torch.randn(4096, 1024, device=gpu) * 0.02).to(torch.bfloat16)
    small = torch.randn(5000, device=gpu)
    ref_w, ref_s = w.clone(), small.clone()
    pending = Snapshot.async_take(str(tmp_path / "s"), {"sd": StateDict(w=w, s=small)},
                                  compression="hsz1")
    w.add_(1.0)
    small.mul_(0)
    pending.wait()
    out = StateDict(w=torch.zeros_like(w), s=torch.zeros_like(small))
    Snapshot(str(tmp_path / "s")).restore({"sd": out})
    assert torch.equal(out["w"], ref_w) and torch.equal(out["s"], ref_s)


def _fsdp_compressed_worker(path):
    from torch.distributed.device_mesh import init_device_mesh

    from hipsnapshot.models.llama import LlamaConfig, build_fsdp_llama

    mesh = init_device_mesh("cuda", (1,))
    model = build_fsdp_llama(LlamaConfig.tiny(), torch.device("cuda:0"), torch.bfloat16,
                             mesh=mesh)
    ref = {k: v.full_tensor().clone() for k, v in model.state_dict().items()}
    Snapshot.take(path, {"model": model}, compression="hsz1")
    with torch.no_grad():
        for p in model.parameters():
            p.to_local().zero_()
    Snapshot(path).restore({"model": model})
    for k, v in model.state_dict().items():
        assert torch.equal(v.full_tensor(), ref[k]), k


def test_gpu_compressed_fsdp2_single_rank(gpu, tmp_path):
    run_distributed(_fsdp_compressed_worker, 1, str(tmp_path / "f"), backend="nccl")


@pytest.mark.parametrize("save_ws,load_ws", [(2, 3)])
def test_multirank_gpu_compressed_gloo(gpu, tmp_path, save_ws, load_ws):
    p = str(tmp_path / "mrc")
    run_distributed(_multirank_gpu_worker, save_ws, p, "save", "hsz1", backend="gloo")
    run_distributed(_multirank_gpu_worker, load_ws, p, "load", "hsz1", backend="gloo")


@pytest.mark.parametrize("compression", ["none", "hsz1"])
def test_take_orders_after_pending_default_stream_work(gpu, tmp_path, compression):
    """Copy streams are non-blocking: a take issued while the trainer's default
    (null) stream is still busy must wait for that work, not read stale HBM."""
    torch.cuda.synchronize()
    a = torch.randn(4096, 4096, device=gpu)
    big = torch.zeros(4096, 4096, device=gpu)
    small = [torch.zeros(1000, device=gpu) for _ in range(8)]
    for _ in range(30):  # keep the default stream busy for a while
        a = torch.tanh(a @ a) * 0.5
    big.copy_(a)
    for s in small:
        s.copy_(a[0, :1000])
    Snapshot.take(str(tmp_path / "s"), {"sd": StateDict(big=big, small=small)},
                  compression=compression)  # no synchronize before the take
    got = Snapshot(str(tmp_path / "s")).read_object("0/sd/big")
    assert torch.equal(got, big.cpu())
    assert torch.equal(Snapshot(str(tmp_path / "s")).read_object("0/sd/small/3"),
                       small[3].cpu())
    # restore into targets whose zeroing is still queued on the default stream
    out_big = torch.ones_like(big)
    out_small = [torch.ones(1000, device=gpu) for _ in range(8)]
    for _ in range(10):
        a = torch.tanh(a @ a) * 0.5
    out_big.mul_(0)
    for s in out_small:
        s.mul_(0)
    Snapshot(str(tmp_path / "s")).restore({"sd": StateDict(big=out_big, small=out_small)})
    assert torch.equal(out_big, big) and all(torch.equal(x, small[0]) for x in out_small)


def test_copy_workspace_ordered_after_busy_default_stream(gpu):
    """A staging thread gathers slabs (copy-kernel workspaces come from torch's
    caching allocator on the default stream) while the main thread keeps that
    stream busy, frees small tensors with kernels still queued and reuses the
    memory: no queued kernel may see its inputs overwritten."""
    import threading

    from hipsnapshot.engine import staging

    stop = threading.Event()
    errors = []

    def worker():
        try:
            ts = [torch.randn(1000 + i, device=gpu) for i in range(8)]
            refs = torch.cat([t.cpu() for t in ts])
            offs = [sum((1000 + j) * 4 for j in range(i)) for i in range(8)]
            total = offs[-1] + (1007) * 4
            while not stop.is_set():
                st = staging.wait_ready(staging.gather_to_host(list(zip(ts, offs)), total, []))
                got = torch.frombuffer(bytearray(st.view), dtype=torch.float32)
                st.release()
                if not torch.equal(got, refs):
                    errors.append("slab bytes differ")
                    return
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))

    th = threading.Thread(target=worker)
    th.start()
    a = torch.randn(2048, 2048, device=gpu)
    results = []
    try:
        for i in range(300):
            a = torch.tanh(a @ a)  # keeps the default stream backed up
            x = torch.full((65536,), float(i), device=gpu)
            y = x * 2
            del x  # freed while `x * 2` may still be queued
            results.append((i, y))
        torch.cuda.synchronize()
    finally:
        stop.set()
        th.join()
    assert not errors, errors
    for i, y in results:
        assert torch.all(y == 2.0 * i), i


# ---- SDMA device -> host engine (csrc/hsdma.hip) ----------------------------

def test_sdma_d2h_sees_kernel_writes_just_made(gpu):
    """The SDMA engine reads HBM behind the L2: bytes a kernel wrote on the
    producer stream right before the copy must arrive (system-scope release)."""
    if native.sdma_engines(0) == 0:
        pytest.skip("ROCr reports no SDMA engine")
    n = (96 << 20) + 4096 + 17
    pb = native.PinnedBuffer(n)
    host = torch.frombuffer(pb.view, dtype=torch.uint8)[:n]
    s = torch.cuda.Stream()
    src = torch.empty(n, dtype=torch.uint8, device=gpu)
    try:
        for val in (3, 250, 77):
            with torch.cuda.stream(s):
                src.fill_(val)
                src[12345:99999].random_(0, 255)
            # no host sync: the copy must order itself after the stream
            native.sdma_d2h(0, pb.ptr, src.data_ptr(), n, s)
            assert torch.equal(host, src.cpu()), val
        for k in (1, 2, 3):  # split over several engines
            with torch.cuda.stream(s):
                src.random_(0, 255)
            native.sdma_d2h(0, pb.ptr, src.data_ptr(), n, s, max_engines=k)
            assert torch.equal(host, src.cpu()), k
    finally:
        pb.release()


@pytest.mark.parametrize("compression", ["none", "hsz1"])
def test_snapshot_with_sdma_d2h(gpu, tmp_path, compression):
    if native.sdma_engines(0) == 0:
        pytest.skip("ROCr reports no SDMA engine")
    sd = _compressible_state(gpu)
    ref = _clone_state(sd)
    with override_knob("D2H_ENGINE", "sdma"):
        Snapshot.take(str(tmp_path / "s"), {"sd": sd}, compression=compression)
        pending = Snapshot.async_take(str(tmp_path / "a"), {"sd": sd}, compression=compression)
        for k, v in sd.items():  # mutate after unblock: must not leak
            if isinstance(v, torch.Tensor):
                v.zero_()
        pending.wait()
    for p in ("s", "a"):
        out = {k: (torch.zeros_like(v) if isinstance(v, torch.Tensor) else
                   [torch.zeros_like(x) for x in v] if isinstance(v, list) else v)
               for k, v in ref.items()}
        out = StateDict(**out)
        Snapshot(str(tmp_path / p)).restore({"sd": out})
        torch.cuda.synchronize()
        assert_state_dict_eq({k: out[k] for k in ref}, ref)


# ---- take-plan reuse on device-resident state (engine/plan_cache.py) ---------

def test_plan_reuse_gpu_sync_and_async(gpu, tmp_path):
    from hipsnapshot.engine import plan_cache

    plan_cache.clear()
    h0 = plan_cache.stats["hits"]
    sd = _compressible_state(gpu)
    sd["host"] = torch.randn(3000)           # per-take host leaf next to cached ones
    refs = []
    for i, mode in enumerate(["sync", "sync", "async", "async", "sync"]):
        for k, v in sd.items():
            if isinstance(v, torch.Tensor):
                v.add_(1)
            elif isinstance(v, list):
                for x in v:
                    x.add_(1)
        sd["step"] = i
        refs.append(_clone_state(sd))
        path = str(tmp_path / f"p{i}")
        if mode == "sync":
            Snapshot.take(path, {"sd": sd}, compression="hsz1")
        else:
            p = Snapshot.async_take(path, {"sd": sd}, compression="hsz1")
            for k, v in sd.items():  # after unblock: must not leak
                if isinstance(v, torch.Tensor):
                    v.mul_(-3)
            p.wait()
            for k, v in refs[-1].items():
                if isinstance(v, torch.Tensor):
                    sd[k].copy_(v)
    # sync plan reused by takes 1 and 4, async plan by take 3
    assert plan_cache.stats["hits"] - h0 == 3
    for i, ref in enumerate(refs):
        out = StateDict(**{k: (torch.zeros_like(v) if isinstance(v, torch.Tensor) else
                               [torch.zeros_like(x) for x in v] if isinstance(v, list) else v)
                           for k, v in ref.items()})
        Snapshot(str(tmp_path / f"p{i}")).restore({"sd": out})
        torch.cuda.synchronize()
        assert_state_dict_eq({k: out[k] for k in ref}, ref)
    plan_cache.clear()


def test_reused_async_plan_full_then_partial_then_full_freeze(gpu, tmp_path, monkeypatch):
    """Warm async takes reset only the stagers their freeze does not
    re-point (plan_cache.lookup(defer_reset=True)): a take whose freeze is
    partial (HBM short) must stage the rest from the live tensors -- not
    from the previous take's arena -- and the next full freeze must cover
    everything again.  Tensors change right after every unblock."""
    from hipsnapshot.engine import hbm_staging, plan_cache

    plan_cache.clear()
    hbm_staging.release_hbm_arena()
    torch.manual_seed(3)
    sd = StateDict(**{f"big{i}": torch.randn(1 << 20, device=gpu) for i in range(6)},
                   **{f"small{i}": torch.randn(1000 + i, device=gpu) for i in range(8)})
    reserve = knobs.hbm_staging_reserve_bytes()
    real_info = torch.cuda.mem_get_info
    real_freeze = hbm_staging.freeze_device_state
    frozen_bytes = []

    def spy(write_reqs, plan=None, **kw):
        out = real_freeze(write_reqs, plan, **kw)
        frozen_bytes.append(sum(out.values()))
        return out

    hbm_staging.freeze_device_state = spy
    refs = []
    try:
        for i, mode in enumerate(["full", "full", "partial", "full"]):
            for v in sd.values():
                v.add_(1)
            refs.append({k: v.clone() for k, v in sd.items()})
            if mode == "partial":
                # the kept arena (which the previous take's stagers still
                # point into) counts as busy -- a drain still reading it --
                # so this take freezes into a new, smaller arena: room for
                # ~2 of the 4 MiB tensors
                for k in hbm_staging._kept.values():
                    k[1] = True
                monkeypatch.setattr(torch.cuda, "mem_get_info",
                                    lambda d=None: (reserve + (9 << 20), real_info(d)[1]))
                monkeypatch.setattr(hbm_staging, "_cached_unused", lambda d: 0)
            else:
                monkeypatch.setattr(torch.cuda, "mem_get_info", real_info)
                monkeypatch.undo()
            p = Snapshot.async_take(str(tmp_path / f"a{i}"), {"sd": sd})
            for v in sd.values():  # after unblock: must not leak into the snapshot
                v.mul_(-7)
            p.wait()
            for k in hbm_staging._kept.values():
                k[1] = False
            for k, v in refs[-1].items():
                sd[k].copy_(v)
    finally:
        monkeypatch.undo()
        hbm_staging.freeze_device_state = real_freeze
    # the third take froze part of the state, the others all of it
    assert frozen_bytes[2] < frozen_bytes[1] == frozen_bytes[3], frozen_bytes
    assert frozen_bytes[2] > 0, frozen_bytes
    assert plan_cache.stats["hits"] >= 3
    for i, ref in enumerate(refs):
        out = StateDict(**{k: torch.zeros_like(v) for k, v in ref.items()})
        Snapshot(str(tmp_path / f"a{i}")).restore({"sd": out})
        torch.cuda.synchronize()
        for k in ref:
            assert torch.equal(out[k], ref[k]), (i, k)
    plan_cache.clear()


@pytest.mark.parametrize("where", ["submit", "wait", "blocking"])
def test_sdma_failure_falls_back_to_blit(gpu, tmp_path, monkeypatch, where):
    """An SDMA copy that fails to start (submit / blocking call) or that the
    engine reports failed (wait) is redone with hipMemcpyAsync, and SDMA is
    switched off for the device."""
    from hipsnapshot.engine import staging

    def broken(*a, **k):
        raise native.HipError("injected SDMA failure")

    if where == "submit":
        monkeypatch.setattr(native, "sdma_d2h_submit", broken)
    elif where == "wait":
        real_wait = native.sdma_wait

        def wait_then_fail(h):
            real_wait(h)  # the copy must be over before its buffer is reused
            raise native.HipError("injected SDMA failure")

        monkeypatch.setattr(native, "sdma_wait", wait_then_fail)
    else:
        monkeypatch.setattr(knobs.TUNING, "async_dma", False)
        monkeypatch.setattr(native, "sdma_d2h", broken)
    monkeypatch.setattr(staging, "_sdma_ok", {0: True})
    sd = StateDict(w=torch.randn(3000, 1000, device=gpu), b=torch.randn(77, device=gpu))
    ref = {k: v.clone() for k, v in sd.items()}
    with override_knob("D2H_ENGINE", "sdma"):
        Snapshot.take(str(tmp_path / "s"), {"sd": sd})
    assert staging._sdma_ok[0] is False
    out = StateDict(w=torch.zeros_like(ref["w"]), b=torch.zeros_like(ref["b"]))
    Snapshot(str(tmp_path / "s")).restore({"sd": out})
    torch.cuda.synchronize()
    assert torch.equal(out["w"], ref["w"]) and torch.equal(out["b"], ref["b"])


# ---- hs64 blob checksums hashed in HBM (hs_hash64, ops/checksum.py) ----------

@pytest.mark.parametrize("n,off", [(0, 0), (1, 0), (7, 3), (8, 0), (24, 0), (4095, 1),
                                   (1 << 20, 0), ((1 << 20) + 8, 8), ((64 << 20) + 13, 5),
                                   ((256 << 20) + 8, 0), ((256 << 20) + 3, 8)])
def test_gpu_hash_matches_host_definition(gpu, n, off):
    from hipsnapshot.ops import checksum

    x = torch.randint(0, 256, (n + off,), dtype=torch.uint8, device=gpu)
    torch.cuda.synchronize()
    h = checksum.device_hash_start(0, 0, x.data_ptr() + off, n)
    got = checksum.device_hash_result(0, 0, h, n)
    host = x.cpu().numpy()[off:]
    assert got == checksum.hs64_of(host)
    if n <= (1 << 20):
        assert got == checksum.hs64_reference(host.tobytes())


@pytest.mark.parametrize("compression", ["none", "hsz1"])
def test_gpu_take_checksums_hashed_on_device_and_verify(gpu, tmp_path, compression, monkeypatch):
    from hipsnapshot.ops import checksum

    calls = []
    real = checksum.device_hash_result

    def counting(dev, slot, handle, nbytes):
        calls.append(nbytes)
        return real(dev, slot, handle, nbytes)

    monkeypatch.setattr(checksum, "device_hash_result", counting)
    sd = _compressible_state(gpu)
    s = Snapshot.take(str(tmp_path / "s"), {"sd": sd}, compression=compression)
    assert calls, "no blob was hashed on the GPU"
    rep = s.verify()
    assert rep.ok and rep.checked == rep.blobs, rep
    calls.clear()
    from hipsnapshot.engine import native_drain

    drained = []
    real_drain = native_drain.drain
    monkeypatch.setattr(native_drain, "drain",
                        lambda reqs, st, *a: drained.append(len(reqs)) or real_drain(reqs, st, *a))
    a = Snapshot.async_take(str(tmp_path / "a"), {"sd": sd}, compression=compression).wait()
    # raw frozen blobs are hashed on the GPU by the native drain (hsg_hash64
    # from C++), the rest through the Python staging path
    assert calls or drained
    assert a.verify().ok
    # flip one byte of the largest blob: the GPU-recorded hash must catch it
    root = str(tmp_path / "s")
    files = [os.path.join(d, f) for d, _, fs in os.walk(root) for f in fs
             if not os.path.relpath(os.path.join(d, f), root).startswith(".snapshot")]
    victim = max(files, key=os.path.getsize)
    with open(victim, "r+b") as f:
        f.seek(7)
        b = f.read(1)
        f.seek(7)
        f.write(bytes([b[0] ^ 1]))
    assert s.verify().mismatched == [os.path.relpath(victim, root)]


@pytest.mark.parametrize("batching", [True, False])
def test_gpu_compressed_restore_with_split_head_read(gpu, tmp_path, monkeypatch, batching):
    """Whole HSZ1 blobs read as a head and the rest: the head's frames go up
    by H2D while the rest is read, then one decode -- direct into the target
    (plain tensors) and through the scratch + region copy (slabs)."""
    from hipsnapshot.knobs import override_is_batching_disabled

    monkeypatch.setattr(knobs.TUNING, "read_head_bytes", 64 * 1024)
    torch.manual_seed(5)
    sd = StateDict(
        w=(torch.randn(1500, 1000, device=gpu) * 0.02).to(torch.bfloat16),
        v=(torch.randn(700, 900, device=gpu) * 0.02).to(torch.bfloat16),
        f=torch.randn(400, 1000, device=gpu) * 1e-2,
    )
    ref = {k: v.clone() for k, v in sd.items()}
    with override_is_batching_disabled(not batching), \
            override_slab_size_threshold_bytes(8 << 20):
        Snapshot.take(str(tmp_path / "s"), {"sd": sd}, compression="hsz1")
        for v in sd.values():
            v.zero_()
        Snapshot(str(tmp_path / "s")).restore({"sd": sd})
    torch.cuda.synchronize()
    for k, v in ref.items():
        assert torch.equal(sd[k], v), k


# ---- native drain of an async take (csrc/hsdrain.cpp) ---------------------------

def _drain_state(gpu):
    torch.manual_seed(11)
    big = torch.randn(3000, 4099, device=gpu)                        # own blob, 49 MB
    col = torch.randn(2048, 3000, device=gpu, dtype=torch.bfloat16)[:, 7:2007]  # strided view
    small = [torch.randn(1000 + 37 * i, device=gpu, dtype=torch.bfloat16) for i in range(40)]
    odd = torch.randint(0, 255, (12345,), dtype=torch.uint8, device=gpu)  # slab gap after it
    return StateDict(big=big, col=col, small=small, odd=odd, step=3)


def _blob_files(root):
    out = {}
    for r, _, fs in os.walk(root):
        for f in fs:
            p = os.path.join(r, f)
            rel = os.path.relpath(p, root)
            if not rel.startswith("."):
                out[rel] = open(p, "rb").read()
    return out


def _odirect_dir(tmp_path):
    """A directory whose filesystem takes O_DIRECT (tmpfs does not)."""
    import shutil
    import uuid

    for d in (tmp_path, os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                     ".odirect_tmp", uuid.uuid4().hex)):
        os.makedirs(d, exist_ok=True)
        try:
            fd = os.open(os.path.join(d, "probe"), os.O_WRONLY | os.O_CREAT | os.O_DIRECT)
            os.close(fd)
            os.unlink(os.path.join(d, "probe"))
            return str(d), (lambda: None) if d == tmp_path else (lambda: shutil.rmtree(d))
        except OSError:
            continue
    pytest.skip("no filesystem with O_DIRECT")


@pytest.mark.parametrize("fsync,direct", [(False, False), (True, False), (False, True)])
def test_native_drain_matches_python_drain(gpu, tmp_path, fsync, direct, monkeypatch):
    """The native drain writes byte-identical blobs (slab gaps zero, strided
    views packed) to the Python drain -- buffered, fdatasync'd or O_DIRECT
    (tail blocks padded, then trimmed) -- records the same hs64 checksums,
    is consistent under in-place updates right after async_take, and is
    actually the path that ran."""
    from hipsnapshot.engine import native_drain
    from hipsnapshot.verify import verify_snapshot

    cleanup = lambda: None  # noqa: E731
    if direct:
        tmp_path, cleanup = _odirect_dir(tmp_path)
        import pathlib

        tmp_path = pathlib.Path(tmp_path)
        monkeypatch.setenv("HIPSNAPSHOT_FS_DIRECT_IO", "1")
    try:
        _native_vs_python_drain(gpu, tmp_path, fsync, monkeypatch, native_drain,
                                verify_snapshot)
    finally:
        cleanup()


def _native_vs_python_drain(gpu, tmp_path, fsync, monkeypatch, native_drain, verify_snapshot):

    calls = []
    orig = native_drain.drain
    monkeypatch.setattr(native_drain, "drain",
                        lambda reqs, st, *a: calls.append(len(reqs)) or orig(reqs, st, *a))
    sd = _drain_state(gpu)
    ref = {k: (v.clone() if torch.is_tensor(v) else [t.clone() for t in v]
               if isinstance(v, list) else v) for k, v in sd.items()}
    opts = {"fsync": fsync}
    p_nat = str(tmp_path / "native")
    # big (49 MB) and col (8 MB, strided) become their own blobs, the rest
    # goes into device slabs with gaps
    monkeypatch.setenv("HIPSNAPSHOT_SLAB_SIZE_THRESHOLD_BYTES_OVERRIDE", str(4 << 20))
    pending = Snapshot.async_take(p_nat, {"sd": sd}, storage_options=opts)
    sd["big"].add_(1.0)  # after the freeze on the same stream
    for t in sd["small"]:
        t.zero_()
    pending.wait()
    assert calls and calls[0] >= 3, calls  # 2 tensors + >= 1 slab
    with override_knob("NATIVE_DRAIN", "0"):
        for k, v in ref.items():  # same values for the Python drain
            if torch.is_tensor(v):
                sd[k].copy_(v)
            elif isinstance(v, list):
                for a, b in zip(sd[k], v):
                    a.copy_(b)
        p_py = str(tmp_path / "python")
        Snapshot.async_take(p_py, {"sd": sd}, storage_options=opts).wait()
    assert len(calls) == 1  # the knob disabled it
    a, b = _blob_files(p_nat), _blob_files(p_py)
    assert a.keys() == b.keys()
    diff = {}
    for k in a:
        if a[k] != b[k]:
            x = np.frombuffer(a[k], np.uint8)
            y = np.frombuffer(b[k], np.uint8)
            n = min(x.size, y.size)
            bad = np.nonzero(x[:n] != y[:n])[0]
            diff[k] = (x.size, y.size, int(bad[0]) if bad.size else None, int(bad.size))
    assert not diff, diff
    import json
    ca = json.load(open(os.path.join(p_nat, ".snapshot_checksums", "0")))["blobs"]
    cb = json.load(open(os.path.join(p_py, ".snapshot_checksums", "0")))["blobs"]
    assert ca == cb and len(ca) == len(a)
    assert verify_snapshot(p_nat).ok
    out = StateDict(big=torch.zeros_like(ref["big"]), col=torch.zeros_like(ref["col"]),
                    small=[torch.zeros_like(t) for t in ref["small"]],
                    odd=torch.zeros_like(ref["odd"]), step=0)
    Snapshot(p_nat).restore({"sd": out})
    assert torch.equal(out["big"], ref["big"]) and torch.equal(out["col"], ref["col"])
    assert torch.equal(out["odd"], ref["odd"]) and out["step"] == 3
    for x, y in zip(out["small"], ref["small"]):
        assert torch.equal(x, y)


def test_native_drain_rewrite_trims_and_async_codec_policy(gpu, tmp_path):
    """An async take into a path whose files are larger (an earlier take of a
    bigger state) leaves exactly the new bytes; compression='hsz1' async
    takes drain the frozen device state raw by default (natively) and encode
    with knobs.TUNING.async_device_codec = "same"."""
    p = str(tmp_path / "s")
    w = torch.randn(4096, 1024, device=gpu)
    with override_slab_size_threshold_bytes(1 << 20):  # w is its own blob
        Snapshot.take(p, {"sd": StateDict(w=torch.randn(8192, 1024, device=gpu))})
        size_before = os.path.getsize(os.path.join(p, "0", "sd", "w"))
        Snapshot.async_take(p, {"sd": StateDict(w=w)}, compression="hsz1").wait()
    assert os.path.getsize(os.path.join(p, "0", "sd", "w")) == w.numel() * 4 < size_before
    e = Snapshot(p).get_manifest()["0/sd/w"]
    assert getattr(e, "codec", None) is None
    got = torch.zeros_like(w)
    Snapshot(p).restore({"sd": StateDict(w=got)})
    assert torch.equal(got, w)
    with override_knob("ASYNC_DEVICE_CODEC", "same"):
        Snapshot.async_take(p + "_c", {"sd": StateDict(w=w)}, compression="hsz1").wait()
    assert Snapshot(p + "_c").get_manifest()["0/sd/w"].codec is not None
    got.zero_()
    Snapshot(p + "_c").restore({"sd": StateDict(w=got)})
    assert torch.equal(got, w)


def test_kept_hbm_arena_reused_and_never_shared(gpu, tmp_path):
    """The async-take arena is kept between takes and reused once its drain
    finished; a take that starts while a drain still reads it gets its own;
    every snapshot holds its own values; release_hbm_arena frees it."""
    from hipsnapshot import release_hbm_arena
    from hipsnapshot.engine import hbm_staging

    release_hbm_arena()
    w = torch.randn(4096, 4096, device=gpu)
    refs = []
    Snapshot.async_take(str(tmp_path / "a0"), {"sd": StateDict(w=w)}).wait()
    refs.append(w.clone())
    first = hbm_staging._kept[0][0].data_ptr()
    w.add_(1.0)
    p1 = Snapshot.async_take(str(tmp_path / "a1"), {"sd": StateDict(w=w)})
    refs.append(w.clone())
    assert hbm_staging._kept[0][0].data_ptr() == first and hbm_staging._kept[0][1]
    w.add_(1.0)  # a second take while the first drain may still run
    p2 = Snapshot.async_take(str(tmp_path / "a2"), {"sd": StateDict(w=w)})
    refs.append(w.clone())
    p1.wait()
    p2.wait()
    assert not hbm_staging._kept[0][1]
    for i, ref in enumerate(refs):
        got = torch.zeros_like(w)
        Snapshot(str(tmp_path / f"a{i}")).restore({"sd": StateDict(w=got)})
        assert torch.equal(got, ref), i
    del p1, p2, got
    import gc

    gc.collect()
    torch.cuda.synchronize()
    before = torch.cuda.memory_allocated(gpu)
    freed = release_hbm_arena()
    assert freed >= w.numel() * 4 and not hbm_staging._kept
    # the memory really goes back: no cached plan's stager pins the arena
    assert before - torch.cuda.memory_allocated(gpu) >= freed, (before, freed)


def test_rebalance_blob_bytes_two_slabs_busy_stream(gpu):
    """Two device slabs gathered for xGMI moves off one rank while the stream
    is still busy: each launch's descriptor stage must stay alive until the
    stream passes it, so both buffers hold exactly their members' bytes."""
    from hipsnapshot.io.batcher import GPUBatchedBufferStager, batch_write_requests
    from hipsnapshot.io.preparer import prepare_write
    from hipsnapshot.parallel.rebalance import _blob_bytes

    torch.manual_seed(0)
    ts = [torch.randn(4096 + 13 * i, device=gpu) for i in range(12)]
    entries, wrs = [], []
    for i, t in enumerate(ts):
        e, w = prepare_write(t, f"sd/t{i}", rank=0, replicated=False)
        entries.append(e)
        wrs += w
    _, out = batch_write_requests(entries, wrs, slab_size_threshold_bytes=4 * 4096 * 4)
    slabs = [w for w in out if isinstance(w.buffer_stager, GPUBatchedBufferStager)]
    assert len(slabs) >= 2
    a = torch.randn(2048, 2048, device=gpu)
    for _ in range(20):  # queue work ahead of the gathers
        a = a @ a
        a /= a.norm()
    got = [_blob_bytes(w) for w in slabs]
    torch.cuda.current_stream().synchronize()
    for w, (buf, _keep) in zip(slabs, got):
        st = w.buffer_stager
        want = torch.zeros(st.total, dtype=torch.uint8, device=gpu)
        for (lo, hi), m in st.members:
            src = m._source_view().reshape(-1).view(torch.uint8)
            want[lo:lo + src.numel()] = src
        assert torch.equal(buf, want)


@pytest.mark.parametrize("comp", ["none", "hsz1"])
def test_native_restore_verify_flags_flipped_byte(gpu, tmp_path, comp):
    """restore(verify=True) into HBM: the native job hashes every whole blob
    in HBM right after its upload.  A byte flipped in a raw blob, or in an
    HSZ1 blob's low-byte plane (which the frame checks do not cover), fails
    the verified restore; the default restore is unchanged (and wrong)."""
    from hipsnapshot.engine import native_restore
    from hipsnapshot.ops import codec
    from hipsnapshot.ops.native import CorruptBlobError

    p = str(tmp_path / "s")
    torch.manual_seed(7)
    w = (torch.randn(2048, 1024, device=gpu) * 0.02).to(torch.bfloat16)
    b = torch.randn(3000, device=gpu)
    with override_slab_size_threshold_bytes(1 << 20):  # w is its own blob
        Snapshot.take(p, {"sd": StateDict(w=w, b=b)}, compression=comp)
    snap = Snapshot(p)
    entry = snap.get_manifest()["0/sd/w"]
    assert bool(entry.codec) == (comp == "hsz1")
    ow, ob = torch.zeros_like(w), torch.zeros_like(b)
    snap.restore({"sd": StateDict(w=ow, b=ob)}, verify=True)
    torch.cuda.synchronize()
    assert torch.equal(ow, w) and torch.equal(ob, b)
    assert native_restore.last_stats.get("items", 0) >= 1  # the native job ran
    blob = os.path.join(p, entry.location)
    if comp == "hsz1":
        from hipsnapshot.utils.test_utils import low_byte_offset

        with open(blob, "rb") as f:
            off = low_byte_offset(f.read())
    else:
        off = (entry.byte_range[0] if entry.byte_range else 0) + 4097
    with open(blob, "r+b") as f:
        f.seek(off)
        c = f.read(1)
        f.seek(off)
        f.write(bytes([c[0] ^ 0x20]))
    ow.zero_()
    Snapshot(p).restore({"sd": StateDict(w=ow, b=ob)})
    torch.cuda.synchronize()
    assert not torch.equal(ow, w)
    with pytest.raises(CorruptBlobError, match=entry.location):
        Snapshot(p).restore({"sd": StateDict(w=torch.zeros_like(w), b=torch.zeros_like(b))},
                            verify=True)
