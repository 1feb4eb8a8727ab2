import numpy as np
import pytest
import torch

from hipsnapshot.format.serialization import (
    ALL_SUPPORTED_DTYPES,
    BUFFER_PROTOCOL_SUPPORTED_DTYPES,
    contiguous_cpu_bytes_view,
    dtype_to_element_size,
    dtype_to_string,
    string_to_dtype,
    tensor_from_bytes,
    torch_load_from_bytes,
    torch_save_as_bytes,
)
from hipsnapshot.utils.test_utils import rand_tensor, tensor_eq


@pytest.mark.parametrize("dtype", ALL_SUPPORTED_DTYPES, ids=str)
def test_dtype_tables(dtype):
    assert string_to_dtype(dtype_to_string(dtype)) == dtype
    if dtype not in (torch.qint32, torch.qint8, torch.quint8):
        assert dtype_to_element_size(dtype) == torch.empty(0, dtype=dtype).element_size()


@pytest.mark.parametrize("dtype", BUFFER_PROTOCOL_SUPPORTED_DTYPES, ids=str)
def test_buffer_protocol_roundtrip(dtype):
    t = rand_tensor([7, 5], dtype)
    mv = contiguous_cpu_bytes_view(t)
    assert mv.nbytes == t.numel() * t.element_size()
    back = tensor_from_bytes(bytes(mv), dtype, [7, 5])
    assert tensor_eq(back, t)
    # non-contiguous input is packed in C order
    tt = t.t()
    back = tensor_from_bytes(bytes(contiguous_cpu_bytes_view(tt)), dtype, [5, 7])
    assert tensor_eq(back, tt.contiguous())


def test_little_endian_layout_matches_numpy():
    t = torch.arange(6, dtype=torch.int32)
    assert bytes(contiguous_cpu_bytes_view(t)) == np.arange(6, dtype="<i4").tobytes()
    b = torch.tensor([1.0, -2.5], dtype=torch.bfloat16)
    raw = bytes(contiguous_cpu_bytes_view(b))
    assert raw == b.view(torch.int16).numpy().astype("<i2").tobytes()


@pytest.mark.parametrize("dtype", [torch.complex64, torch.qint8, torch.quint8, torch.qint32],
                         ids=str)
def test_torch_save_roundtrip_weights_only(dtype):
    t = rand_tensor([4, 4], dtype)
    back = torch_load_from_bytes(torch_save_as_bytes(t), trusted=False)
    assert tensor_eq(back, t)


def test_zero_size():
    t = torch.empty(0, 3)
    assert contiguous_cpu_bytes_view(t).nbytes == 0
    assert tensor_from_bytes(b"", torch.float32, [0, 3]).shape == (0, 3)


def test_per_tensor_qtensor_codec():
    from hipsnapshot.format.serialization import (per_tensor_qtensor_as_bytes,
                                                  per_tensor_qtensor_from_bytes)

    for dt in (torch.qint8, torch.quint8, torch.qint32):
        q = torch.quantize_per_tensor(torch.rand(5, 7) * 5, 0.05, 3, dt)
        back = per_tensor_qtensor_from_bytes(per_tensor_qtensor_as_bytes(q))
        assert tensor_eq(back, q) and back.q_scale() == q.q_scale()


def test_per_channel_qtensor_codec():
    from hipsnapshot.format.serialization import (per_channel_qtensor_as_bytes,
                                                  per_channel_qtensor_from_bytes)

    x = torch.rand(6, 4, 3) * 4
    q = torch.quantize_per_channel(x, torch.rand(4) + 0.01, torch.randint(0, 10, (4,)), 1,
                                   torch.quint8)
    back = per_channel_qtensor_from_bytes(per_channel_qtensor_as_bytes(q))
    assert torch.equal(back.int_repr(), q.int_repr())
    assert torch.equal(back.q_per_channel_scales(), q.q_per_channel_scales().double())
    assert back.q_per_channel_axis() == 1
