"""Randomised end-to-end round trips: seeded random app states (nested
dicts / lists, every supported dtype, 0-d / empty / non-contiguous tensors,
odd keys, Python objects) saved with random options (compression, batching,
small chunk / slab thresholds, take vs async_take) and restored IN PLACE into
zeroed copies, then compared exactly; ``read_object`` of a random leaf too.

The CPU cases run everywhere; the GPU cases put most tensors on ``cuda:0``,
so the SDMA staging, gather / scatter kernels, HSZ1 coder and native restore
all run under the same random mix.  ``HS_E2E_SEEDS`` / ``HS_E2E_GPU_SEEDS``
widen the search (defaults 16 / 24).
"""

import os
import random

import pytest
import torch

from hipsnapshot import Snapshot, StateDict, knobs
from hipsnapshot.format.serialization import SUPPORTED_QUANTIZED_DTYPES
from hipsnapshot.utils.test_utils import all_dtypes, assert_state_dict_eq, rand_tensor

KEYS = ["w", "bias", "a/b", "%x", "7", "layer.0", "+1", "01", "é"]


def _tensor(rng: random.Random, device: str):
    dtype = rng.choice(all_dtypes())
    if dtype in SUPPORTED_QUANTIZED_DTYPES:
        device = "cpu"  # quantized tensors live on the CPU
    r = rng.random()
    if r < 0.08:
        shape = []
    elif r < 0.14:
        shape = [0, rng.randint(1, 4)]
    elif r < 0.24:
        shape = [rng.randint(40_000, 400_000)]  # several chunks / its own slab
    elif r < 0.28 and device != "cpu":
        shape = [rng.randint(1 << 21, 1 << 24)]  # many ring slots of the native engines
    else:
        shape = [rng.randint(1, 33) for _ in range(rng.randint(1, 3))]
    t = rand_tensor(shape, dtype, device="cpu")
    if device != "cpu":
        t = t.to(device)
    if t.dim() >= 2 and not t.is_quantized and rng.random() < 0.3:
        t = t.transpose(0, 1)  # non-contiguous leaf
    elif t.dim() >= 1 and t.shape[0] > 2 and not t.is_quantized and rng.random() < 0.2:
        t = t[1: t.shape[0] - 1]  # a view at a storage offset of a larger tensor
    return t


def _value(rng: random.Random, device: str, depth: int = 0):
    r = rng.random()
    if r < 0.6 or depth >= 2:
        return _tensor(rng, device)
    if r < 0.75:
        return {rng.choice(KEYS) + str(i): _value(rng, device, depth + 1)
                for i in range(rng.randint(0, 3))}
    if r < 0.85:
        return [_value(rng, device, depth + 1) for _ in range(rng.randint(0, 3))]
    return rng.choice([3, -7, "text", None, 2.5, [1, "a"], {"k": (1, 2)}])


def _random_state(rng: random.Random, device: str) -> dict:
    return {f"{rng.choice(KEYS)}_{i}": _value(rng, device) for i in range(rng.randint(1, 8))}


def _blank(v):
    """A same-structure copy whose tensors are zeroed (same strides) and whose
    objects differ: what a restore must overwrite."""
    if isinstance(v, torch.Tensor):
        if v.is_quantized:
            return torch.quantize_per_tensor(torch.zeros(v.shape), 1.0, 0, v.dtype)
        z = torch.empty_strided(v.shape, v.stride(), dtype=v.dtype, device=v.device)
        z.zero_()
        return z
    if isinstance(v, dict):
        return {k: _blank(x) for k, x in v.items()}
    if isinstance(v, list):
        return [_blank(x) for x in v]
    return "placeholder"


FLOAT_CASTS = [torch.float32, torch.bfloat16, torch.float16, torch.float64]


def _cross(v, rng: random.Random):
    """(target, expected): like ``_blank``, but a floating tensor's target
    may have another float dtype and / or live on the other device.  Same
    dtype and shape: restored in place, across devices.  Another dtype:
    TorchSnapshot's rule -- the value is read into a new tensor of the saved
    dtype, which a ``StateDict`` takes as is (``nn.Module.load_state_dict``
    would then cast it into its parameter; DTensor targets are cast in place
    by the scatter, ``tests/test_dist_random.py``)."""
    if isinstance(v, torch.Tensor):
        if v.is_quantized or not v.is_floating_point() or v.dtype not in FLOAT_CASTS:
            return _blank(v), v
        dtype = rng.choice(FLOAT_CASTS) if rng.random() < 0.4 else v.dtype
        dev = v.device
        if rng.random() < 0.3:
            dev = torch.device("cpu") if v.is_cuda else torch.device("cuda", 0)
        z = torch.zeros(v.shape, dtype=dtype, device=dev)
        return z, (v.to(device=dev) if dtype == v.dtype else v)
    if isinstance(v, dict):
        pairs = {k: _cross(x, rng) for k, x in v.items()}
        return {k: a for k, (a, _b) in pairs.items()}, {k: b for k, (_a, b) in pairs.items()}
    if isinstance(v, list):
        pairs = [_cross(x, rng) for x in v]
        return [a for a, _b in pairs], [b for _a, b in pairs]
    return "placeholder", v


def _random_tuning(rng: random.Random) -> dict:
    """Engine constants far from their defaults: tiny rings that wrap many
    times per blob, one slot, one copy in flight, no idle pool kept."""
    slot = rng.choice([1 << 20, 4 << 20, 128 << 20])
    return {
        "restore_slot_bytes": slot,
        "restore_slots": rng.choice([1, 2, 3, 6]),
        "restore_first_bytes": min(slot, rng.choice([1 << 20, 16 << 20])),
        "restore_piece_bytes": min(slot, rng.choice([64 << 10, 1 << 20, 4 << 20])),
        "read_head_bytes": rng.choice([256 << 10, 16 << 20]),
        "restore_keep_bytes": rng.choice([0, (2 << 30) + (256 << 20)]),
        "drain_slot_bytes": rng.choice([1 << 20, 8 << 20, 64 << 20]),
        "drain_slots": rng.choice([1, 2, 16]),
        "dma_inflight": rng.choice([1, 2, 8]),
        "stage_threads": rng.choice([1, 4]),
        "plan_cache": rng.random() < 0.5,
    }


def _round_trip(tmp_path, seed: int, device: str, tuning: bool = False,
                cross: bool = False) -> None:
    rng = random.Random(seed)
    if tuning:
        with knobs.override_tuning(**_random_tuning(random.Random(seed + 7))):
            return _round_trip(tmp_path, seed, device, cross=cross)
    state = _random_state(rng, device)
    compression = rng.choice(["none", "hsz1", "hsz1+host"])
    batching = rng.random() < 0.7
    chunk = rng.choice([None, 64 << 10, 1 << 20])
    slab = rng.choice([None, 16 << 10, 256 << 10])
    use_async = rng.random() < 0.4
    case = dict(seed=seed, compression=compression, batching=batching, chunk=chunk, slab=slab,
                use_async=use_async)
    path = os.path.join(str(tmp_path), f"s{seed}")
    with knobs.override_is_batching_disabled(not batching):
        ctx = [knobs.override_max_chunk_size_bytes(chunk) if chunk else None,
               knobs.override_slab_size_threshold_bytes(slab) if slab else None]
        for c in ctx:
            if c is not None:
                c.__enter__()
        try:
            app = {"app": StateDict(**state)}
            if use_async:
                snap = Snapshot.async_take(path, app, compression=compression).wait()
            else:
                snap = Snapshot.take(path, app, compression=compression)
            if cross:
                tgt, expect = _cross(state, random.Random(seed + 11))
            else:
                tgt, expect = _blank(state), state
            target = {"app": StateDict(**tgt)}
            Snapshot(path).restore(target, verify=rng.random() < 0.3)
        finally:
            for c in reversed(ctx):
                if c is not None:
                    c.__exit__(None, None, None)
    assert_state_dict_eq(dict(target["app"]), expect, f"case {case}")
    # read_object of top-level tensor leaves: into a fresh buffer, and into a
    # zeroed obj_out under a random memory budget (tiled reads)
    from hipsnapshot.format.flatten import encode_key

    for key, v in state.items():
        if not isinstance(v, torch.Tensor):
            continue
        p = f"0/app/{encode_key(key)}"
        assert_state_dict_eq(snap.read_object(p), v, f"read_object {p} {case}")
        if v.is_quantized or v.numel() == 0:
            continue
        budget = rng.choice([None, 4096, 100_000])
        out = _blank(v)
        snap.read_object(p, obj_out=out, memory_budget_bytes=budget,
                         verify=rng.random() < 0.3)
        assert_state_dict_eq(out, v, f"read_object {p} budget {budget} {case}")


@pytest.mark.parametrize("seed", range(int(os.environ.get("HS_E2E_SEEDS", "16"))))
def test_random_state_round_trip_cpu(tmp_path, seed):
    _round_trip(tmp_path, seed, "cpu")


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(100, 100 + int(os.environ.get("HS_E2E_GPU_SEEDS", "24"))))
def test_random_state_round_trip_gpu(tmp_path, gpu, seed):
    _round_trip(tmp_path, seed, "cuda:0")


@pytest.mark.parametrize("qscheme", ["tensor", "channel0", "channel1"])
def test_chunked_quantized_restores_its_qparams(tmp_path, monkeypatch, qscheme):
    """A chunked quantized tensor (the reference chunks them; hipsnapshot now
    writes them whole) restores into a destination with other qparams, and
    reads back without one.  Found by the random round trips: chunks were
    copied into views of the destination, which kept its old scale."""
    from hipsnapshot.io import chunked, preparer

    def always_chunk(obj, path, is_async, prepare_func, serializer, max_chunk, max_shard):
        return chunked.ChunkedTensorIOPreparer.prepare_write(
            storage_path=path, tensor=obj,
            chunking_instruction=chunked.ChunkedTensorIOPreparer.chunk_tensor(
                obj, chunk_sz_bytes=64), is_async_snapshot=is_async)

    monkeypatch.setitem(preparer._WRITERS, "tensor", always_chunk)
    base = torch.rand(10, 6) * 10
    if qscheme == "tensor":
        q = torch.quantize_per_tensor(base, 0.1, 10, torch.quint8)
        blank = torch.quantize_per_tensor(torch.zeros(10, 6), 1.0, 0, torch.quint8)
    else:
        axis = int(qscheme[-1])
        n = base.shape[axis]
        q = torch.quantize_per_channel(base, torch.rand(n) * 0.1 + 0.05,
                                       torch.randint(0, 5, (n,)), axis, torch.quint8)
        blank = torch.quantize_per_channel(torch.zeros(10, 6), torch.ones(n),
                                           torch.zeros(n, dtype=torch.long), axis, torch.quint8)
    path = str(tmp_path / "s")
    snap = Snapshot.take(path, {"app": StateDict(q=q)})
    assert snap.get_manifest()["0/app/q"].type == "ChunkedTensor"
    target = {"app": StateDict(q=blank)}
    Snapshot(path).restore(target)
    assert_state_dict_eq(dict(target["app"]), {"q": q})
    assert_state_dict_eq({"q": snap.read_object("0/app/q")}, {"q": q})


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(500, 500 + int(os.environ.get("HS_E2E_GPU_SEEDS", "24"))))
def test_random_state_round_trip_gpu_engine_tuning(tmp_path, gpu, seed):
    """The same under random engine constants (``_random_tuning``): the native
    drain's and restore's rings with 1 MiB slots, 1 slot, 1 DMA in flight."""
    _round_trip(tmp_path, seed, "cuda:0", tuning=True)


@pytest.mark.parametrize("seed", range(500, 506))
def test_random_state_round_trip_cpu_engine_tuning(tmp_path, seed):
    _round_trip(tmp_path, seed, "cpu", tuning=True)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(700, 700 + int(os.environ.get("HS_E2E_GPU_SEEDS", "24"))))
def test_random_state_round_trip_gpu_cross_dtype_device(tmp_path, gpu, seed):
    """Restore targets of another float dtype and / or on the other device
    (GPU -> host, host -> GPU): cast kernels and H2D / D2H on restore."""
    _round_trip(tmp_path, seed, "cuda:0", cross=True)


def _alias_case(tmp_path, seed: int, device: str) -> None:
    """Entries that share storage: a tied weight listed twice, overlapping
    slices and a transpose of one base tensor (slab gather, HBM freeze and
    in-place restore must each see consistent bytes)."""
    rng = random.Random(seed)
    n = rng.randint(8, 600)
    base = torch.randn(n, 16, device=device).to(rng.choice([torch.float32, torch.bfloat16]))
    a0, a1 = sorted(rng.sample(range(n), 2))
    b0 = rng.randrange(a0, a1 + 1)
    def views(t):
        return {"tied_a": t, "tied_b": t, "s1": t[a0:a1 + 1], "s2": t[b0:],
                "tr": t.t(), "col": t[:, 3:9]}
    state = views(base)
    comp = rng.choice(["none", "hsz1"])
    path = os.path.join(str(tmp_path), f"al{seed}")
    ref = base.clone()
    if rng.random() < 0.5:
        pend = Snapshot.async_take(path, {"sd": StateDict(**state)}, compression=comp)
        base.add_(1)  # after the take: not in the snapshot
        pend.wait()
    else:
        Snapshot.take(path, {"sd": StateDict(**state)}, compression=comp)
    fresh = torch.zeros_like(base)
    out = StateDict(**views(fresh))
    Snapshot(path).restore({"sd": out})
    assert torch.equal(fresh, ref), (seed, device, comp)
    for k, v in views(ref).items():
        assert torch.equal(out[k], v), (seed, k)


@pytest.mark.parametrize("seed", range(6))
def test_aliased_entries_round_trip_cpu(tmp_path, seed):
    _alias_case(tmp_path, seed, "cpu")


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(100, 100 + int(os.environ.get("HS_E2E_GPU_SEEDS", "24"))))
def test_aliased_entries_round_trip_gpu(tmp_path, gpu, seed):
    _alias_case(tmp_path, seed, "cuda:0")
