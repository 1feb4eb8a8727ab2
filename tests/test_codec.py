"""HSZ1 lossless codec: format, round trip, compressibility (CPU)."""

import numpy as np
import pytest

from hipsnapshot import knobs
import torch

from hipsnapshot.ops import codec


def _bytes(t: torch.Tensor) -> bytes:
    return t.contiguous().view(torch.uint8).numpy().tobytes()


@pytest.mark.parametrize("dtype,w", [(torch.bfloat16, 2), (torch.float16, 2),
                                     (torch.float32, 4)])
@pytest.mark.parametrize("n", [1, 7, 4096, 300_001])
def test_reference_roundtrip(dtype, w, n):
    x = (torch.randn(n) * 0.02).to(dtype)
    raw = _bytes(x)
    blob = codec.encode_reference(raw, w, frame_bytes=64 * 1024)
    assert codec.decode_reference(blob) == raw
    h = codec.parse_header(blob)
    assert h.logical_size == len(raw) and h.offsets[-1] == len(blob)
    assert all(o % 16 == 0 for o in h.offsets)


def test_compression_ratio_on_weight_like_data():
    x = (torch.randn(2_000_000) / 64).to(torch.bfloat16)
    raw = _bytes(x)
    blob = codec.encode_reference(raw, 2)
    ratio = len(blob) / len(raw)
    # mode 2: 8 raw bits + ~2.7 Huffman bits per bf16, within 1 % of the entropy bound
    assert 0.66 < ratio < 0.68, ratio
    assert set(codec.frame_modes(blob)) == {2}
    hi = np.frombuffer(raw, dtype=np.uint8)[1::2]
    p = np.bincount(hi, minlength=256) / hi.size
    ent = -(p[p > 0] * np.log2(p[p > 0])).sum()
    assert ratio < (8 + ent) / 16 * 1.012
    y = torch.randn(1_000_000) * 1e-3
    blob = codec.encode_reference(_bytes(y), 4)
    # fp32: 24 raw bits + ~2.7 Huffman bits per element (mode 1 would be 0.876)
    assert 0.83 < len(blob) / (4 * y.numel()) < 0.845
    assert set(codec.frame_modes(blob)) == {2}


def test_fp32_mode2_with_tail_native_matches_reference():
    y = torch.randn(8000) * 0.02
    raw = _bytes(y) + b"\x01\x02\x03"  # 3-byte tail after 8000 elements
    fb = 32016  # one frame holding the whole 32003-byte blob
    blob = codec.encode_reference(raw, 4, frame_bytes=fb)
    assert codec.frame_modes(blob) == [2]
    assert codec.decode_reference(blob) == raw
    assert codec.encode_cpu(raw, 4, fb).tobytes() == blob
    assert codec.decode_cpu(blob).tobytes() == raw
    # a corrupt lane table that points past the frame is rejected, not read
    h = codec.parse_header(blob)
    bad = bytearray(blob)
    tab = h.offsets[0] + codec.FRAME_HEADER_BYTES + 3 * 8000
    bad[tab: tab + 2] = (0xFFFF).to_bytes(2, "little")
    with pytest.raises(RuntimeError):
        codec.decode_cpu(bytes(bad))


def test_incompressible_frames_stored_raw():
    rnd = np.random.default_rng(0).integers(0, 256, 200_000, dtype=np.uint8).tobytes()
    blob = codec.encode_reference(rnd, 2, frame_bytes=16 * 1024)
    assert codec.decode_reference(blob) == rnd
    h = codec.parse_header(blob)
    modes = {blob[h.offsets[i]] for i in range(h.n_frames)}
    assert modes == {0}
    assert len(blob) <= codec.max_encoded_bytes(len(rnd), 16 * 1024)


def test_mixed_blob_and_odd_lengths():
    # slab-like: bf16 weights, fp32 norm, padding, odd tail
    parts = [_bytes((torch.randn(40_000) * 0.02).to(torch.bfloat16)),
             _bytes(torch.ones(1000)), bytes(256), b"\x01\x02\x03"]
    raw = b"".join(parts)
    for fb in (1024, 4096, 65536):
        blob = codec.encode_reference(raw, 2, frame_bytes=fb)
        assert codec.decode_reference(blob) == raw


def test_escape_heavy_frame_falls_back():
    # 20 distinct high bytes evenly spread: > MAX_ESCAPES escapes -> raw frame
    hi = np.repeat(np.arange(20, dtype=np.uint8), 3000)
    el = np.stack([np.zeros_like(hi), hi], 1).reshape(-1)
    blob = codec.encode_reference(el.tobytes(), 2, frame_bytes=len(el))
    h = codec.parse_header(blob)
    assert blob[h.offsets[0]] == 0 and codec.decode_reference(blob) == el.tobytes()


def test_huffman_lengths_rules():
    # prefix-free and complete for ordinary histograms
    lens = codec.huffman_lengths([50, 30, 10, 10] + [0] * 12)
    assert lens[:4] == [1, 2, 3, 3] and sum(2.0 ** -x for x in lens if x) == 1.0
    # ties go to the lower index (deterministic across implementations)
    assert codec.huffman_lengths([5, 5, 5, 5] + [0] * 12)[:4] == [2, 2, 2, 2]
    # one used index -> 1 bit; nothing used -> nothing
    assert codec.huffman_lengths([0, 7] + [0] * 14)[1] == 1
    assert codec.huffman_lengths([0] * 16) == [0] * 16
    # Fibonacci-like counts would need 15 bits: limited to HUFF_MAX_LEN, Kraft <= 1
    fib = [1, 1]
    for _ in range(14):
        fib.append(fib[-1] + fib[-2])
    lens = codec.huffman_lengths(fib)
    assert max(lens) == codec.HUFF_MAX_LEN
    assert sum(2.0 ** -x for x in lens) <= 1.0
    # canonical codes are prefix-free and the LUT inverts them
    lut = codec.decode_table(lens)
    codes = codec.canonical_codes(lens)
    for c in range(16):
        assert lut[codes[c]] == c | (lens[c] << 8)


def test_mode2_frames_and_skewed_histograms():
    # a near-constant high byte (1 dominant index, long codes for the rest)
    g = np.random.default_rng(3)
    hi = np.full(65536, 0x3C, dtype=np.uint8)
    hi[g.integers(0, hi.size, 300)] = g.integers(0x30, 0x40, 300)
    el = np.stack([g.integers(0, 256, hi.size, dtype=np.uint8), hi], 1).reshape(-1)
    raw = el.tobytes() + b"\x07"  # odd tail byte
    blob = codec.encode_reference(raw, 2, frame_bytes=len(raw) - 1)
    assert codec.frame_modes(blob)[0] == 2
    assert codec.decode_reference(blob) == raw
    assert codec.decode_cpu(blob).tobytes() == raw
    assert codec.encode_cpu(raw, 2, len(raw) - 1).tobytes() == blob
    # fewer groups than lanes (most lane streams empty) still round-trips
    small = _bytes((torch.randn(4096) * 0.02).to(torch.bfloat16))
    b2 = codec.encode_reference(small, 2, frame_bytes=len(small))
    assert codec.decode_reference(b2) == small and codec.decode_cpu(b2).tobytes() == small


def test_length_limited_huffman_frame_native_matches_reference():
    from hipsnapshot.utils.test_utils import hsz_deep_tree_frame

    raw = hsz_deep_tree_frame()
    blob = codec.encode_reference(raw, 2, frame_bytes=len(raw))
    o = codec.parse_header(blob).offsets[0]
    lens = [(blob[o + 24 + j // 2] >> (4 * (j % 2))) & 15 for j in range(16)]
    assert codec.frame_modes(blob) == [2] and max(lens) == codec.HUFF_MAX_LEN
    assert codec.decode_reference(blob) == raw
    assert codec.encode_cpu(raw, 2, len(raw)).tobytes() == blob
    assert codec.decode_cpu(blob).tobytes() == raw


def test_version1_blobs_still_decode():
    import struct

    raw = _bytes((torch.randn(50_000) * 0.02).to(torch.bfloat16))
    blob = bytearray(codec.encode_reference(raw, 2, frame_bytes=16 * 1024))
    if set(codec.frame_modes(bytes(blob))) <= {0, 1}:
        struct.pack_into("<I", blob, 4, 1)
        assert codec.decode_reference(bytes(blob)) == raw
    raw8 = _bytes(torch.randn(20_000, dtype=torch.float64) * 0.02)
    v1 = bytearray(codec.encode_reference(raw8, 8, frame_bytes=16 * 1024))  # w=8: modes 0/1
    assert 1 in codec.frame_modes(bytes(v1)) and 2 not in codec.frame_modes(bytes(v1))
    struct.pack_into("<I", v1, 4, 1)
    assert codec.decode_reference(bytes(v1)) == raw8 and codec.decode_cpu(bytes(v1)).tobytes() == raw8


def test_frames_covering():
    h = codec.Header(logical_size=1000, elem_width=2, frame_bytes=256, n_frames=4,
                     offsets=[0] * 5)
    assert h.frames_covering(0, 1000) == (0, 4)
    assert h.frames_covering(255, 257) == (0, 2)
    assert h.frames_covering(512, 513) == (2, 3)
    assert h.frame_range(3) == (768, 1000)


@pytest.mark.parametrize("w", [1, 2, 4, 8])
@pytest.mark.parametrize("n", [0, 5, 65_536, 1_000_003])
def test_native_cpu_codec_matches_reference(w, n):
    g = torch.Generator().manual_seed(n + w)
    x = (torch.randn(n // 2 + 1, generator=g) * 0.02).to(torch.bfloat16)
    raw = _bytes(x)[:n]
    fb = 64 * 1024
    ref = codec.encode_reference(raw, w, fb)
    nat = codec.encode_cpu(raw, w, fb, nthreads=4)
    assert nat.tobytes() == ref
    assert codec.decode_cpu(ref).tobytes() == raw


def test_validate_offsets_rejects_corrupt_table():
    raw = _bytes((torch.randn(100_000) * 0.02).to(torch.bfloat16))
    blob = bytearray(codec.encode_reference(raw, 2, 16 * 1024))
    h = codec.parse_header(blob)
    import struct

    struct.pack_into("<Q", blob, codec.HEADER_BYTES + 8 * 3, h.offsets[3] + 10 ** 9)
    with pytest.raises(ValueError):
        codec.decode_cpu(bytes(blob))


# ---- end to end through Snapshot (host tensors, C++ codec) ------------------------

@pytest.fixture
def host_compression(monkeypatch):
    # the takes below ask for compression="hsz1+host" (host tensors too);
    # takes without compression= must stay uncompressed
    monkeypatch.delenv("HIPSNAPSHOT_COMPRESSION", raising=False)


def _weights(seed=0):
    g = torch.Generator().manual_seed(seed)
    return {
        "big_bf16": (torch.randn(700, 1000, generator=g) * 0.02).to(torch.bfloat16),
        "fp32": torch.randn(300, 300, generator=g) * 1e-2,
        "small": torch.randn(10, generator=g),
        "ints": torch.randint(0, 100, (50_000,), generator=g),
        "fp16": (torch.randn(100_000, generator=g) * 0.1).to(torch.float16),
    }


@pytest.mark.parametrize("batching", [True, False])
def test_snapshot_compressed_roundtrip(tmp_path, host_compression, batching):
    import os

    from hipsnapshot import Snapshot, StateDict
    from hipsnapshot.knobs import override_is_batching_disabled

    src = _weights()
    with override_is_batching_disabled(not batching):
        snap = Snapshot.take(str(tmp_path / "s"), {"sd": StateDict(**src)}, compression="hsz1+host")
        man = snap.get_manifest()
        assert man["0/sd/big_bf16"].codec["name"] == "hsz1"
        assert man["0/sd/big_bf16"].codec["w"] == 2
        if not batching:
            assert man["0/sd/ints"].codec is None  # integers stay raw
            f = tmp_path / "s" / man["0/sd/big_bf16"].location
            assert os.path.getsize(f) < 0.8 * 700 * 1000 * 2
        out = StateDict(**{k: torch.zeros_like(v) for k, v in src.items()})
        Snapshot(str(tmp_path / "s")).restore({"sd": out})
        for k, v in src.items():
            assert torch.equal(out[k], v), k
        # read_object: whole tensor, into a differently-typed target, with budget
        got = Snapshot(str(tmp_path / "s")).read_object("0/sd/big_bf16")
        assert torch.equal(got, src["big_bf16"])
        same = torch.zeros_like(src["big_bf16"])
        got = Snapshot(str(tmp_path / "s")).read_object("0/sd/big_bf16", obj_out=same,
                                                        memory_budget_bytes=1 << 16)
        assert got is same and torch.equal(same, src["big_bf16"])
        # a narrowed (non-contiguous) in-place target of the fp32 entry
        big = torch.zeros(300, 600)
        view = big[:, 100:400]
        Snapshot(str(tmp_path / "s")).read_object("0/sd/fp32", obj_out=view)
        assert torch.equal(view, src["fp32"]) and big[:, :100].abs().sum() == 0


def test_snapshot_compressed_chunked_and_metadata_compat(tmp_path, host_compression):
    import json

    from hipsnapshot import Snapshot, StateDict
    from hipsnapshot.knobs import override_max_chunk_size_bytes

    t = (torch.randn(1000, 300) * 0.02).to(torch.bfloat16)
    with override_max_chunk_size_bytes(100_000):
        Snapshot.take(str(tmp_path / "c"), {"sd": StateDict(t=t)}, compression="hsz1+host")
    md = json.loads((tmp_path / "c" / ".snapshot_metadata").read_text())
    ent = md["manifest"]["0/sd/t"]
    assert ent["type"] == "ChunkedTensor" and len(ent["chunks"]) > 3
    assert all(c["tensor"]["codec"]["name"] == "hsz1" for c in ent["chunks"])
    out = StateDict(t=torch.zeros_like(t))
    Snapshot(str(tmp_path / "c")).restore({"sd": out})
    assert torch.equal(out["t"], t)
    # uncompressed snapshots carry no codec key at all (reference-compatible)
    Snapshot.take(str(tmp_path / "u"), {"sd": StateDict(t=t)})
    md = json.loads((tmp_path / "u" / ".snapshot_metadata").read_text())
    assert "codec" not in json.dumps(md)


def test_snapshot_compressed_dtensor_resharding(tmp_path, host_compression):
    from hipsnapshot.utils.test_utils import run_distributed

    run_distributed(_dtensor_worker, 2, str(tmp_path / "d"), "save")
    run_distributed(_dtensor_worker, 3, str(tmp_path / "d"), "load")


def _dtensor_worker(path: str, mode: str) -> None:
    import os

    import torch.distributed as dist
    from torch.distributed.device_mesh import init_device_mesh
    from torch.distributed.tensor import Shard, distribute_tensor

    from hipsnapshot import Snapshot, StateDict

    mesh = init_device_mesh("cpu", (dist.get_world_size(),))
    torch.manual_seed(0)
    full = (torch.randn(640, 96) * 0.02).to(torch.bfloat16)
    if mode == "save":
        d = distribute_tensor(full, mesh, [Shard(0)])
        Snapshot.take(path, {"sd": StateDict(w=d)}, compression="hsz1+host")
    else:
        d = distribute_tensor(torch.zeros_like(full), mesh, [Shard(1)])
        Snapshot(path).restore({"sd": StateDict(w=d)})
        assert torch.equal(d.full_tensor(), full)


def test_ratio_holds_for_trained_weights_and_adam_state():
    """The high-byte entropy of TRAINED weights and AdamW moments is as low as
    at init (the ratio is not an artefact of random-init data)."""
    torch.manual_seed(0)
    m = torch.nn.Sequential(torch.nn.Linear(128, 512), torch.nn.GELU(), torch.nn.Linear(512, 128))
    opt = torch.optim.AdamW(m.parameters(), lr=3e-3)
    x_all = torch.randn(2048, 128)
    w_t = torch.randn(128, 128) / 12
    for _ in range(150):
        x = x_all[torch.randint(0, 2048, (128,))]
        loss = ((m(x) - torch.tanh(x @ w_t)) ** 2).mean()
        opt.zero_grad()
        loss.backward()
        opt.step()
    st = opt.state[m[0].weight]
    for name, t, bound in [("weight", m[0].weight, 0.70), ("exp_avg", st["exp_avg"], 0.70),
                           ("exp_avg_sq", st["exp_avg_sq"], 0.62)]:
        raw = _bytes(t.detach().to(torch.bfloat16))
        blob = codec.encode_cpu(raw, 2, 64 * 1024)
        assert len(blob) / len(raw) < bound, (name, len(blob) / len(raw))
        assert codec.decode_cpu(blob.tobytes()).tobytes() == raw


# ---- whole blobs read as a head and the rest (knobs.get_read_head_bytes) ----------

@pytest.mark.parametrize("batching", [True, False])
def test_compressed_restore_with_split_head_read(tmp_path, host_compression, monkeypatch,
                                                 batching):
    """Blobs larger than twice the head are read as two requests; the consumer
    decodes once the rest has arrived (host path: decode_host waits)."""
    from hipsnapshot import Snapshot, StateDict
    from hipsnapshot.knobs import override_is_batching_disabled
    from hipsnapshot.storage import fs as fs_mod

    monkeypatch.setattr(knobs.TUNING, "read_head_bytes", 64 * 1024)
    ranges = []
    orig = fs_mod.FSStoragePlugin.read

    async def spy(self, read_io):
        ranges.append(read_io.byte_range)
        await orig(self, read_io)

    monkeypatch.setattr(fs_mod.FSStoragePlugin, "read", spy)
    src = _weights(3)
    with override_is_batching_disabled(not batching):
        Snapshot.take(str(tmp_path / "s"), {"sd": StateDict(**src)}, compression="hsz1+host")
        out = StateDict(**{k: torch.zeros_like(v) for k, v in src.items()})
        Snapshot(str(tmp_path / "s")).restore({"sd": out})
    for k, v in src.items():
        assert torch.equal(out[k], v), k
    assert (0, 64 * 1024) in ranges  # a head read happened
    assert any(r is not None and r[0] == 64 * 1024 for r in ranges)  # and its rest


def test_compressed_restore_fails_when_rest_read_fails(tmp_path, host_compression, monkeypatch):
    """A failing read of a blob's rest fails the restore (no hang, no decode of
    bytes that never arrived)."""
    from hipsnapshot import Snapshot, StateDict
    from hipsnapshot.storage import fs as fs_mod

    src = {"big_bf16": _weights(4)["big_bf16"]}
    Snapshot.take(str(tmp_path / "s"), {"sd": StateDict(**src)}, compression="hsz1+host")
    monkeypatch.setattr(knobs.TUNING, "read_head_bytes", 64 * 1024)
    orig = fs_mod.FSStoragePlugin.read

    async def flaky(self, read_io):
        if read_io.byte_range is not None and read_io.byte_range[0] == 64 * 1024:
            raise OSError(5, "injected read failure")
        await orig(self, read_io)

    monkeypatch.setattr(fs_mod.FSStoragePlugin, "read", flaky)
    out = StateDict(big_bf16=torch.zeros_like(src["big_bf16"]))
    with pytest.raises(OSError, match="injected"):
        Snapshot(str(tmp_path / "s")).restore({"sd": out})
