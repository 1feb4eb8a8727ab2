"""Plan-time choice of which blobs are stored HSZ1-compressed (opt-in).

``Snapshot.take(..., compression="hsz1")`` (or ``HIPSNAPSHOT_COMPRESSION=hsz1``)
marks every blob whose bytes are produced on the GPU and are mostly floating
point: plain tensors / chunks / shard pieces of bf16, fp16, fp32, fp64, and
device slabs whose payload is mostly such tensors.  The choice is recorded in
each member's ``TensorEntry.codec`` before the manifest is gathered, so the
metadata always describes what the stagers will write.  Host (CPU) tensors are
written raw: encoding them would cost host memory bandwidth, which is the
scarce resource a compressed checkpoint is meant to save.

See ``ops/codec.py`` for the format and ``engine/staging.py`` for where the
GPU encodes before D2H / decodes after H2D.
"""

from __future__ import annotations

from collections import Counter
from typing import List, Optional

import torch

from ..format.serialization import SER
from ..io_types import WriteReq
from ..ops import codec as hsz

CODECS = ("none", "hsz1")
MIN_BLOB_BYTES = 64 * 1024

_ELEM_WIDTH = {torch.bfloat16: 2, torch.float16: 2, torch.float32: 4, torch.float64: 8}


def resolve(compression: Optional[str]) -> str:
    from .. import knobs

    c = (compression or knobs.get_compression()).strip().lower()
    base, _, extra = c.partition("+")
    if base not in CODECS or extra not in ("", "host") or (extra and base == "none"):
        raise ValueError(f"unknown compression {c!r}; expected one of {CODECS} "
                         "(a codec may carry '+host': host tensors too)")
    return base


def host_requested(compression: Optional[str]) -> bool:
    """``"hsz1+host"``: host (CPU) tensors are encoded too (C++ codec)."""
    from .. import knobs

    return (compression or knobs.get_compression()).strip().lower().endswith("+host")


def _info(w: int, blob_bytes: int, frame_bytes: int) -> dict:
    return {"name": hsz.CODEC_NAME, "w": w, "frame_bytes": frame_bytes,
            "blob_bytes": int(blob_bytes)}


def _float_stager(st, include_host: bool) -> Optional[int]:
    from .tensor import TensorBufferStager

    if not isinstance(st, TensorBufferStager):
        return None
    if st.entry.serializer != SER.BUFFER_PROTOCOL or st._tensor_prepare_func:
        return None
    t = st.tensor
    if not t.is_cuda and not include_host:
        return None
    return _ELEM_WIDTH.get(t.dtype)


def plan_compression(write_reqs: List[WriteReq],
                     frame_bytes: int = hsz.DEFAULT_FRAME_BYTES,
                     include_host: Optional[bool] = None) -> int:
    """Mark eligible write requests; returns the number of compressed blobs.

    ``include_host`` (default: ``HIPSNAPSHOT_COMPRESSION=hsz1+host``) also encodes
    host tensors with the C++ codec -- worth it when storage, not host memory
    bandwidth, is the bottleneck (network filesystems, object stores).
    """
    from .. import knobs
    from .batcher import BatchedBufferStager, GPUBatchedBufferStager

    if include_host is None:
        include_host = knobs.compress_host_tensors()
    n = 0
    for wr in write_reqs:
        st = wr.buffer_stager
        if isinstance(st, (GPUBatchedBufferStager, BatchedBufferStager)):
            if isinstance(st, BatchedBufferStager) and not include_host:
                continue
            by_w = Counter()
            for (lo, hi), m in st.members:
                w = _float_stager(m, include_host)
                if w is not None:
                    by_w[w] += hi - lo
            if st.total < MIN_BLOB_BYTES or sum(by_w.values()) * 2 < st.total:
                continue
            info = _info(by_w.most_common(1)[0][0], st.total, frame_bytes)
            st.codec = info
            for _, m in st.members:
                m.entry.codec = info
            n += 1
            continue
        w = _float_stager(st, include_host)
        if w is None:
            continue
        nbytes = st.tensor.numel() * st.tensor.element_size()
        if nbytes < MIN_BLOB_BYTES:
            continue
        info = _info(w, nbytes, frame_bytes)
        st.codec = info
        st.entry.codec = info
        n += 1
    return n
