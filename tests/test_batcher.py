"""Batcher: slab planning, relocation, round trips over dtypes x chunking x
batched/tiled reads (reference strategy: tests/test_batcher.py:232-329)."""

import asyncio

import pytest
import torch

from hipsnapshot.format.serialization import BUFFER_PROTOCOL_SUPPORTED_DTYPES
from hipsnapshot.io.batcher import batch_read_requests, batch_write_requests
from hipsnapshot.io.preparer import prepare_read, prepare_write
from hipsnapshot.io_types import StagedBuffer
from hipsnapshot.knobs import override_max_chunk_size_bytes
from hipsnapshot.utils.test_utils import rand_tensor, tensor_eq


def _write_all(write_reqs):
    loop = asyncio.new_event_loop()
    blobs = {}
    try:
        for wr in write_reqs:
            buf = loop.run_until_complete(wr.buffer_stager.stage_buffer())
            view = buf.view if isinstance(buf, StagedBuffer) else memoryview(buf)
            blobs[wr.path] = bytes(view)
            if isinstance(buf, StagedBuffer):
                buf.release()
    finally:
        loop.close()
    return blobs


def _read_all(read_reqs, blobs):
    loop = asyncio.new_event_loop()
    try:
        for rr in read_reqs:
            data = blobs[rr.path]
            if rr.byte_range is not None:
                data = data[rr.byte_range[0]: rr.byte_range[1]]
            loop.run_until_complete(rr.buffer_consumer.consume_buffer(memoryview(data)))
    finally:
        loop.close()


@pytest.mark.parametrize("chunking", [False, True])
@pytest.mark.parametrize("batched_read", [False, True])
@pytest.mark.parametrize("tiled_read", [False, True])
def test_batched_roundtrip(chunking, batched_read, tiled_read):
    torch.manual_seed(0)
    tensors = {f"sd/t{i}": rand_tensor([(i % 7) + 1, 33], BUFFER_PROTOCOL_SUPPORTED_DTYPES[
        i % len(BUFFER_PROTOCOL_SUPPORTED_DTYPES)]) for i in range(50)}
    entries, wrs = {}, []
    ctx = override_max_chunk_size_bytes(200) if chunking else override_max_chunk_size_bytes(1 << 30)
    with ctx:
        for k, t in tensors.items():
            e, w = prepare_write(t, k, 0, replicated=False)
            entries[k] = e
            wrs += w
    n_before = len(wrs)
    _, batched = batch_write_requests(list(entries.values()), wrs,
                                      slab_size_threshold_bytes=4000, name_prefix="r0")
    assert len(batched) < n_before
    assert all(w.path.startswith("batched/r0_cpu_") for w in batched)
    blobs = _write_all(batched)
    outs = {k: torch.zeros_like(t) for k, t in tensors.items()}
    rrs = []
    for k, e in entries.items():
        r, _ = prepare_read(e, outs[k], buffer_size_limit_bytes=64 if tiled_read else None)
        rrs += r
    if batched_read:
        merged = batch_read_requests(rrs)
        if not tiled_read:
            assert len(merged) == len(batched)  # one read per slab
        rrs = merged
    _read_all(rrs, blobs)
    for k in tensors:
        assert tensor_eq(outs[k], tensors[k]), k


def test_slab_alignment_and_threshold():
    ts = [torch.ones(100, dtype=torch.uint8) for _ in range(10)]
    entries, wrs = [], []
    for i, t in enumerate(ts):
        e, w = prepare_write(t, f"sd/{i}", 0, replicated=False)
        entries.append(e)
        wrs += w
    _, batched = batch_write_requests(entries, wrs, slab_size_threshold_bytes=1000)
    ranges = [e.byte_range for e in entries]
    assert all(r[0] % 256 == 0 for r in ranges)  # 16-B aligned members (256-B slots)
    assert all(r[1] - r[0] == 100 for r in ranges)
    assert len(batched) == 3  # 256*3 + 100 < 1000 <= 256*4: four per slab


def test_large_and_unbatchable_not_slabbed():
    big = torch.zeros(2000, dtype=torch.uint8)
    cplx = torch.zeros(4, dtype=torch.complex64)
    e1, w1 = prepare_write(big, "sd/big", 0, replicated=False)
    e2, w2 = prepare_write(cplx, "sd/c", 0, replicated=False)
    _, batched = batch_write_requests([e1, e2], w1 + w2, slab_size_threshold_bytes=1000)
    assert {w.path for w in batched} == {"0/sd/big", "0/sd/c"}
    assert e1.byte_range is None


def test_merged_read_consuming_cost_counts_merged_buffer():
    ts = {f"sd/{i}": torch.randn(10) for i in range(4)}
    entries, wrs = {}, []
    for k, t in ts.items():
        e, w = prepare_write(t, k, 0, replicated=False)
        entries[k] = e
        wrs += w
    batch_write_requests(list(entries.values()), wrs, slab_size_threshold_bytes=10 ** 6)
    rrs = []
    for e in entries.values():
        rrs += prepare_read(e, None)[0]
    (merged,) = batch_read_requests(rrs)
    lo, hi = merged.byte_range
    assert merged.buffer_consumer.get_consuming_cost_bytes() == (hi - lo) + 4 * 40


def test_slab_tail_taper():
    """The last slabs are closed early so the final (serial, per-file) write of
    a take is short; packing of the bulk follows the threshold."""
    ts = [torch.zeros(5 << 20, dtype=torch.uint8) for _ in range(40)]  # 200 MiB
    entries, wrs = [], []
    for i, t in enumerate(ts):
        e, w = prepare_write(t, f"sd/{i}", 0, replicated=False)
        entries.append(e)
        wrs += w
    _, batched = batch_write_requests(entries, wrs, slab_size_threshold_bytes=64 << 20)
    sizes = [w.buffer_stager.total for w in batched]
    assert max(sizes) < 64 << 20 and sum(sizes) >= 200 << 20
    assert sizes[-1] <= 13 << 20
    # geometric: every slab is at most ~an eighth of what is still to come
    # (plus one tensor), so its write finishes while the rest crosses PCIe
    for i, sz in enumerate(sizes):
        rest = sum(sizes[i:])
        assert sz <= max(64 << 20 if rest > 8 * (64 << 20) else 0, rest // 8 + (5 << 20),
                         (8 << 20) + (5 << 20)), (i, sizes)
    assert sizes == sorted(sizes, reverse=True)
