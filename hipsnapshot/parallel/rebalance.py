"""Per-rank write-load rebalancing over xGMI (opt-in).

The reference's partitioner only balances REPLICATED state
(`/root/reference/torchsnapshot/partitioner.py:42-166`); sharded and per-rank
bytes stay with their owner.  When one rank owns much more device state than
its peers -- TABLE_WISE embedding tables, uneven TP/EP layouts -- its PCIe
link (~56 GB/s of D2H) decides the whole take while the other links idle.

On an MI355X node every GPU pair has a direct xGMI link (~50-150 GB/s), so
``rebalance`` (``HIPSNAPSHOT_REBALANCE=1``, sync takes) moves whole blobs from
the most loaded ranks to the least loaded ones before staging:

1. one all-gather of (device bytes to write, movable blobs as (index, bytes,
   path)) -- movable = raw contiguous-bytes blobs (buffer-protocol tensors,
   no HSZ1 codec, no fp8) and raw device slabs;
2. every rank computes the same plan: repeatedly move the largest blob of
   the most loaded rank that fits in half the gap to the least loaded rank
   (strictly lowers the maximum), until the spread is under
   ``REBALANCE_MIN_GAIN`` of the mean;
3. the blob bytes move device to device with RCCL point-to-point
   (``batch_isend_irecv``: xGMI, no host memory), the receiver stages and
   writes them to the SAME path.  Manifests are unchanged (a blob's
   location does not depend on the writer); its checksum is recorded by the
   rank that wrote it.

CPU tensors can be moved too (``knobs.TUNING.rebalance_host``; tests use
it with gloo).  Async takes keep their blobs: the frozen arena is drained
without collectives.
"""

from __future__ import annotations

import logging
from typing import List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

from .. import knobs
from ..io_types import BufferStager, StagedBuffer, WriteReq
from .comm import Comm

logger = logging.getLogger(__name__)


def _movable(wr: WriteReq, host_ok: bool) -> Optional[int]:
    """Bytes of a blob another rank could write from a raw copy, else None."""
    from ..format.serialization import Serializer
    from ..io.batcher import GPUBatchedBufferStager
    from ..io.tensor import TensorBufferStager

    st = wr.buffer_stager
    if getattr(st, "codec", None) is not None:
        return None
    if isinstance(st, TensorBufferStager):
        t = st.tensor
        if st.entry.serializer != Serializer.BUFFER_PROTOCOL.value or \
                st._tensor_prepare_func is not None or (not t.is_cuda and not host_ok):
            return None
        return t.numel() * t.element_size()
    if isinstance(st, GPUBatchedBufferStager):
        return st.total
    return None


def _device_bytes(wr: WriteReq) -> int:
    from ..io.batcher import GPUBatchedBufferStager
    from ..io.tensor import TensorBufferStager

    st = wr.buffer_stager
    if isinstance(st, TensorBufferStager) and st.tensor.is_cuda:
        return st.get_staging_cost_bytes()
    if isinstance(st, GPUBatchedBufferStager):
        return st.total
    return 0


def plan_moves(loads: Sequence[int], cands: Sequence[Sequence[Tuple[int, int, str]]],
               min_gain: float, max_moves: int) -> List[Tuple[int, int, int, int, str]]:
    """Deterministic greedy: [(src rank, blob index, dst rank, bytes, path)]."""
    loads = list(loads)
    left = [sorted(c, key=lambda x: (-x[1], x[0])) for c in cands]
    mean = sum(loads) / max(len(loads), 1)
    moves = []
    while len(moves) < max_moves:
        hi = max(range(len(loads)), key=lambda r: (loads[r], -r))
        lo = min(range(len(loads)), key=lambda r: (loads[r], r))
        gap = loads[hi] - loads[lo]
        if hi == lo or gap <= min_gain * mean:
            break
        pick = next((c for c in left[hi] if c[1] <= gap // 2 and c[1] > 0), None)
        if pick is None:
            break
        left[hi].remove(pick)
        loads[hi] -= pick[1]
        loads[lo] += pick[1]
        moves.append((hi, pick[0], lo, pick[1], pick[2]))
    return moves


class ReceivedBlobStager(BufferStager):
    """A blob another rank sent over xGMI: its raw bytes in a local buffer."""

    thread_staging = True

    def __init__(self, buf: torch.Tensor) -> None:
        self.buf = buf
        self.codec = None

    async def stage_buffer(self, executor=None):
        return self.stage_buffer_sync()

    def stage_buffer_sync(self) -> StagedBuffer:
        from ..engine import staging

        if self.buf.is_cuda:
            dev = self.buf.device
            return staging.d2h_tensor(self.buf, int(torch.cuda.current_stream(dev).cuda_stream))
        from ..format.serialization import contiguous_cpu_bytes_view

        return StagedBuffer(contiguous_cpu_bytes_view(self.buf), keepalive=self.buf)

    def get_staging_cost_bytes(self) -> int:
        return self.buf.numel()


def _blob_bytes(wr: WriteReq) -> Tuple[torch.Tensor, object]:
    """The blob's exact bytes as one contiguous uint8 tensor on its device,
    plus the keepalive of the gather launch that fills it (its pinned
    descriptor stage and device workspace): hold it until the stream has
    passed the launch, or a later launch reuses the stage block and the
    gather reads ITS descriptors."""
    from ..io.batcher import GPUBatchedBufferStager
    from ..ops import native

    st = wr.buffer_stager
    if isinstance(st, GPUBatchedBufferStager):
        dev = st.members[0][1].tensor.device
        out = torch.zeros(st.total, dtype=torch.uint8, device=dev)  # gaps stay zero
        batch = native.CopyBatch()
        for (lo, _hi), m in st.members:
            t = m._source_view().detach()
            if t.numel():
                batch.add_tensor(t, out.data_ptr() + lo)
        keep = batch.launch(dev.index or 0, int(torch.cuda.current_stream(dev).cuda_stream),
                            sync=False)
        return out, keep
    t = st._source().contiguous()
    return t.reshape(-1).view(torch.uint8), None


def rebalance(write_reqs: List[WriteReq], comm: Comm) -> List[WriteReq]:
    ws = comm.get_world_size()
    if comm.solo() or not knobs.rebalance_enabled():
        return write_reqs
    host_ok = knobs.rebalance_host()
    mine = []
    for i, wr in enumerate(write_reqs):
        n = _movable(wr, host_ok)
        if n:
            mine.append((i, n, wr.path, _device_bytes(wr) > 0))
    load = sum(_device_bytes(wr) for wr in write_reqs)
    if host_ok:
        load += sum(c[1] for c in mine if not c[3])
    gathered: List = [None] * ws
    comm.all_gather_object(gathered, (load, mine))
    cands = [[(c[0], c[1], c[2]) for c in g[1]] for g in gathered]
    on_dev = {(r, c[0]): c[3] for r, g in enumerate(gathered) for c in g[1]}
    moves = plan_moves([g[0] for g in gathered], cands, knobs.rebalance_min_gain(), 4 * ws)
    if not moves:
        return write_reqs
    rank = comm.get_rank()
    logger.info(f"rebalance: {len(moves)} blob(s), "
                f"{sum(m[3] for m in moves) / 1e9:.2f} GB over xGMI")
    sends, recvs, keep, launches, outgoing, incoming = [], [], [], [], set(), []
    for src, idx, dst, n, path in moves:
        if rank == src:
            buf, ka = _blob_bytes(write_reqs[idx])
            keep.append(buf)
            if ka is not None:
                launches.append(ka)
            outgoing.add(idx)
            sends.append((buf, dst))
        elif rank == dst:
            dev = torch.device("cuda", torch.cuda.current_device()) if on_dev[(src, idx)] \
                else torch.device("cpu")
            buf = torch.empty(n, dtype=torch.uint8, device=dev)
            incoming.append((path, buf))
            recvs.append((buf, src))
    if keep and any(b.is_cuda for b in keep):
        # every gather launch (and the producers queued before it on this
        # stream) must be done before a send reads its buffer and before its
        # pinned descriptor stage goes back to the pool
        torch.cuda.current_stream().synchronize()
    launches.clear()
    p2p_exchange(sends, recvs, comm)
    kept = [wr for i, wr in enumerate(write_reqs) if i not in outgoing]
    return kept + [WriteReq(path=p, buffer_stager=ReceivedBlobStager(b)) for p, b in incoming]


def p2p_exchange(sends: Sequence[Tuple[torch.Tensor, int]],
                 recvs: Sequence[Tuple[torch.Tensor, int]], comm: Comm) -> None:
    """Post every send ``(tensor, dst)`` and receive ``(tensor, src)`` (ranks
    relative to ``comm.pg``) and wait for all of them.  RCCL: one
    ``batch_isend_irecv`` group (device buffers over xGMI; no ordering
    deadlock, and a rank may be its own peer); CPU backends: plain
    isend/irecv."""
    pg = comm.pg

    def peer(r: int) -> int:
        return dist.get_global_rank(pg, r) if pg is not dist.group.WORLD else r

    ops = [dist.P2POp(dist.isend, t, peer(d), group=pg) for t, d in sends] + \
          [dist.P2POp(dist.irecv, t, peer(s), group=pg) for t, s in recvs]
    if not ops:
        return
    if "nccl" in str(comm.backend()):
        works = dist.batch_isend_irecv(ops)
    else:
        works = [op.op(op.tensor, op.peer, group=op.group) for op in ops]
    for w in works:
        w.wait()
