"""HSZ1 lossless codec: format, round trip, compressibility (CPU)."""

import numpy as np
import pytest
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
    assert 0.74 < ratio < 0.77, ratio  # 12 bits per bf16 + escapes + headers
    y = torch.randn(1_000_000) * 1e-3
    blob = codec.encode_reference(_bytes(y), 4)
    assert len(blob) / (4 * y.numel()) < 0.88


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
