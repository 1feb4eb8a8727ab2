"""Tensor/chunked preparers: stagers feed consumers directly (no storage).

Mirrors the reference's ``_fulfill_read_reqs_with_write_reqs`` strategy
(tests/test_tensor_io_preparer.py:33-56) on our own API.
"""

import asyncio
from typing import List

import pytest
import torch

from hipsnapshot.format.manifest import TensorEntry
from hipsnapshot.format.serialization import BUFFER_PROTOCOL_SUPPORTED_DTYPES
from hipsnapshot.io.chunked import ChunkedTensorIOPreparer
from hipsnapshot.io.tensor import TensorIOPreparer, tensor_copy
from hipsnapshot.io_types import ReadReq, StagedBuffer, WriteReq
from hipsnapshot.knobs import override_max_chunk_size_bytes
from hipsnapshot.utils.test_utils import all_dtypes, rand_tensor, tensor_eq


def fulfill(write_reqs: List[WriteReq], read_reqs: List[ReadReq]) -> None:
    loop = asyncio.new_event_loop()
    try:
        blobs = {}
        for wr in write_reqs:
            buf = loop.run_until_complete(wr.buffer_stager.stage_buffer())
            view = buf.view if isinstance(buf, StagedBuffer) else memoryview(buf)
            blobs[wr.path] = bytes(view)
            if isinstance(buf, StagedBuffer):
                buf.release()
        for rr in read_reqs:
            data = blobs[rr.path]
            if rr.byte_range is not None:
                data = data[rr.byte_range[0]: rr.byte_range[1]]
            loop.run_until_complete(rr.buffer_consumer.consume_buffer(data))
    finally:
        loop.close()


@pytest.mark.parametrize("dtype", all_dtypes(), ids=str)
def test_roundtrip_all_dtypes(dtype):
    src = rand_tensor([13, 7], dtype)
    entry, wrs = TensorIOPreparer.prepare_write("0/x", src)
    assert entry.shape == [13, 7] and entry.dtype == str(dtype)
    expected = "buffer_protocol" if dtype in BUFFER_PROTOCOL_SUPPORTED_DTYPES else "torch_save"
    assert entry.serializer == expected
    dst = rand_tensor([13, 7], dtype) if not dtype.is_complex else torch.zeros(13, 7, dtype=dtype)
    if dtype in (torch.qint8, torch.quint8, torch.qint32):
        rrs, fut = TensorIOPreparer.prepare_read(entry, dst)
    else:
        rrs, fut = TensorIOPreparer.prepare_read(entry, dst)
        assert fut.obj is dst  # in place
    fulfill(wrs, rrs)
    assert tensor_eq(fut.obj, src)


def test_read_without_obj_out_allocates():
    src = torch.randn(5, 5)
    entry, wrs = TensorIOPreparer.prepare_write("0/x", src)
    rrs, fut = TensorIOPreparer.prepare_read(entry)
    fulfill(wrs, rrs)
    assert torch.equal(fut.obj, src)


def test_shape_mismatch_allocates_new():
    src = torch.randn(5, 5)
    entry, wrs = TensorIOPreparer.prepare_write("0/x", src)
    dst = torch.zeros(4, 4)
    rrs, fut = TensorIOPreparer.prepare_read(entry, dst)
    assert fut.obj is not dst
    fulfill(wrs, rrs)
    assert torch.equal(fut.obj, src)


@pytest.mark.parametrize("shape", [[1000], [997], [31, 29], [4, 5, 6]])
@pytest.mark.parametrize("limit", [1, 64, 1000, 10 ** 9])
def test_tiled_reads(shape, limit):
    src = torch.randn(shape)
    entry, wrs = TensorIOPreparer.prepare_write("0/x", src)
    dst = torch.zeros(shape)
    rrs, fut = TensorIOPreparer.prepare_read(entry, dst, buffer_size_limit_bytes=limit)
    n = src.numel() * 4
    assert len(rrs) == min(src.numel(), -(-n // limit))
    for rr in rrs:
        assert rr.byte_range[1] - rr.byte_range[0] <= max(limit, 4)
    assert rrs[0].byte_range[0] == 0 and rrs[-1].byte_range[1] == n
    fulfill(wrs, rrs)
    assert torch.equal(fut.obj, src)


def test_tiled_read_into_non_contiguous_target():
    src = torch.randn(64, 32)
    entry, wrs = TensorIOPreparer.prepare_write("0/x", src)
    big = torch.zeros(32, 64)
    dst = big.t()  # non-contiguous view with matching shape
    rrs, fut = TensorIOPreparer.prepare_read(entry, dst, buffer_size_limit_bytes=512)
    fulfill(wrs, rrs)
    assert torch.equal(dst, src) and torch.equal(big.t(), src)


def test_write_non_contiguous_and_offset_views():
    base = torch.randn(20, 30)
    for view in (base.t(), base[3:9, 5:25], base[::2, ::3], base[7]):
        entry, wrs = TensorIOPreparer.prepare_write("0/v", view)
        rrs, fut = TensorIOPreparer.prepare_read(entry)
        fulfill(wrs, rrs)
        assert torch.equal(fut.obj, view)


def test_custom_prepare_func_output_is_what_gets_saved():
    src = torch.randn(8, 8)

    def to_half(t, tracing):
        return t.half()

    entry, wrs = TensorIOPreparer.prepare_write("0/x", src, _tensor_prepare_func=to_half)
    assert entry.dtype == "torch.float16"
    rrs, fut = TensorIOPreparer.prepare_read(entry)
    fulfill(wrs, rrs)
    assert fut.obj.dtype == torch.float16 and torch.equal(fut.obj, src.half())


def test_custom_prepare_func_quantize():
    src = torch.rand(16, 16)

    def q(t, tracing):
        return torch.quantize_per_tensor(t, 0.1, 10, torch.qint8)

    entry, wrs = TensorIOPreparer.prepare_write("0/x", src, _tensor_prepare_func=q)
    assert entry.dtype == "torch.qint8" and entry.serializer == "torch_save"
    dst = torch.zeros(16, 16)
    rrs, fut = TensorIOPreparer.prepare_read(entry)
    fulfill(wrs, rrs)
    assert torch.allclose(fut.obj.dequantize(), src, atol=0.06)


def test_prepare_func_shape_change_rejected():
    with pytest.raises(RuntimeError):
        TensorIOPreparer.prepare_write("0/x", torch.randn(4), _tensor_prepare_func=lambda t, tr: t[:2])


FLOATS = [torch.float64, torch.float32, torch.float16, torch.bfloat16]


@pytest.mark.parametrize("src_dtype", FLOATS, ids=str)
@pytest.mark.parametrize("dst_dtype", FLOATS, ids=str)
def test_tensor_copy_float_matrix(src_dtype, dst_dtype):
    src = torch.randn(10, 10).to(src_dtype)
    dst = torch.zeros(10, 10, dtype=dst_dtype)
    tensor_copy(dst, src)
    assert torch.equal(dst, src.to(dst_dtype))


def test_tensor_copy_quantized_to_float_and_requant():
    q = torch.quantize_per_tensor(torch.rand(6, 6), 0.1, 3, torch.qint8)
    f = torch.zeros(6, 6)
    tensor_copy(f, q)
    assert torch.equal(f, q.dequantize())
    q2 = torch.quantize_per_tensor(torch.rand(6, 6), 0.2, 1, torch.qint8)
    tensor_copy(q2, q)
    assert torch.equal(q2.int_repr(), q.int_repr())
    # view with different qparams: dequantize first
    big = torch.quantize_per_tensor(torch.rand(12, 6), 0.05, 0, torch.qint8)
    view = big[:6]
    tensor_copy(view, q)
    assert torch.allclose(big[:6].dequantize(), q.dequantize(), atol=0.05)


@pytest.mark.parametrize("n_rows", [1, 7, 100])
def test_chunking_math(n_rows):
    t = torch.randn(n_rows, 33)
    nbytes = t.numel() * 4
    for chunk in [33 * 4, 1000, nbytes, nbytes * 2]:
        chunks = ChunkedTensorIOPreparer.chunk_tensor(t, chunk_sz_bytes=chunk)
        assert sum(c.sizes[0] for c in chunks) == n_rows
        assert chunks[0].offsets == [0, 0]
        for a, b in zip(chunks, chunks[1:]):
            assert b.offsets[0] == a.offsets[0] + a.sizes[0]


def test_chunked_roundtrip_and_locations():
    t = torch.randn(100, 50)
    with override_max_chunk_size_bytes(4000):
        instr = ChunkedTensorIOPreparer.chunk_tensor(t)
        entry, wrs = ChunkedTensorIOPreparer.prepare_write("0/big", t, instr)
    assert len(entry.chunks) == len(wrs) > 1
    assert entry.chunks[1].tensor.location == f"0/big_{entry.chunks[1].offsets[0]}_0"
    dst = torch.zeros(100, 50)
    rrs, fut = ChunkedTensorIOPreparer.prepare_read(entry, dst)
    assert fut.obj is dst
    fulfill(wrs, rrs)
    assert torch.equal(dst, t)
    rrs, fut = ChunkedTensorIOPreparer.prepare_read(entry, None, buffer_size_limit_bytes=300)
    fulfill(wrs, rrs)
    assert torch.equal(fut.obj, t)


def test_chunked_zero_dim():
    t = torch.tensor(3.5)
    instr = ChunkedTensorIOPreparer.chunk_tensor(t, chunk_sz_bytes=1)
    assert len(instr) == 1 and instr[0].sizes == [1]
