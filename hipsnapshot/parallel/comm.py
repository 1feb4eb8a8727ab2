"""Process-group facade for the planner's metadata collectives.

Reference: `/root/reference/torchsnapshot/pg_wrapper.py:15-89` (``PGWrapper``).
Only small pickled objects travel (paths, keys, entries, write-load plans --
SURVEY 2.5); checkpoint payload never crosses the interconnect.

On MI355X the process group is RCCL (torch backend name ``"nccl"``) over xGMI,
one rank per GPU.  Object collectives stage their bytes on the rank's current
HIP device, so ``Comm`` pins the device once (``torch.cuda.set_device`` is the
caller's job -- we assert it is set to a device this rank owns when the
backend is RCCL).

Ordering: with RCCL every collective (and the frame's host <-> device
copies) runs with a dedicated side stream as the current stream.  ProcessGroup
collectives make the communication stream wait on the CURRENT stream, and a
blocking ``.cpu()`` waits for it too: on the trainer's stream a metadata
all-gather would first wait for every kernel the training step had queued
(torch's own object collectives do exactly that), so ``async_take`` would
only return once the GPU drained the step.  The side stream carries nothing
but these small collectives.

Latency: torch's ``all_gather_object`` is two collectives (sizes, then padded
payload).  ``Comm.all_gather_object`` is ONE collective when every payload
fits a fixed 64 KiB frame (header with the true length + bytes), and falls
back to a second round only for the ranks' overflow -- halving the
latency-bound collective count of a take (10 + K object collectives,
SURVEY 3.5).  Results are identical to torch's.

World size 1: the reference issues every collective whenever a process group
is given (`/root/reference/torchsnapshot/pg_wrapper.py:42-56`).  ``Comm``
skips them for a one-rank group (nothing to exchange) unless
``HIPSNAPSHOT_FORCE_COLLECTIVES=1`` (or ``Comm(pg, force=True)``): then a
one-rank RCCL group runs the same framed all-gather, device broadcast and
device barrier as an N-rank one -- the GPU tests use it so every RCCL code
path has executed on the MI355X before a multi-GPU job relies on it.
"""

from __future__ import annotations

import contextlib
import pickle
import struct
import threading
from typing import Any, Dict, List, Optional

import torch
import torch.distributed as dist

from .. import knobs

_FRAME = 64 * 1024
_HDR = struct.Struct("<q")

_side: Dict[int, "torch.cuda.Stream"] = {}
_side_lock = threading.Lock()


def _side_stream(dev: int) -> "torch.cuda.Stream":
    s = _side.get(dev)
    if s is None:
        with _side_lock:
            s = _side.get(dev)
            if s is None:
                s = _side[dev] = torch.cuda.Stream(device=dev)
    return s


class Comm:
    def __init__(self, pg: Optional[dist.ProcessGroup] = None,
                 force: Optional[bool] = None) -> None:
        if pg is None and dist.is_available() and dist.is_initialized():
            pg = dist.group.WORLD
        self.pg = pg
        self.force = knobs.force_collectives() if force is None else bool(force)

    def solo(self) -> bool:
        """No collective is issued: no process group, or a one-rank group
        outside forced mode.  Callers that skip a collective (or a store
        barrier) at world size 1 must test this, not the world size."""
        return self.pg is None or (not self.force and self.get_world_size() == 1)

    # -- topology ----------------------------------------------------------

    def get_rank(self) -> int:
        return dist.get_rank(group=self.pg) if self.pg is not None else 0

    def get_world_size(self) -> int:
        return dist.get_world_size(group=self.pg) if self.pg is not None else 1

    def backend(self) -> Optional[str]:
        return dist.get_backend(self.pg) if self.pg is not None else None

    def _device(self) -> torch.device:
        be = self.backend()
        if be is not None and "nccl" in str(be):
            return torch.device("cuda", torch.cuda.current_device())
        return torch.device("cpu")

    def _on_side_stream(self):
        """RCCL: run the collective with the side stream as current stream
        (see the module docstring); a no-op for CPU backends."""
        if "nccl" not in str(self.backend()):
            return contextlib.nullcontext()
        return torch.cuda.stream(_side_stream(torch.cuda.current_device()))

    # -- collectives -------------------------------------------------------

    def barrier(self) -> None:
        if self.solo():
            return
        if "nccl" in str(self.backend()):
            with self._on_side_stream():
                dist.barrier(group=self.pg, device_ids=[torch.cuda.current_device()])
        else:
            dist.barrier(group=self.pg)

    def broadcast_object_list(self, obj_list: List[Any], src: int = 0) -> None:
        if self.solo():
            return
        with self._on_side_stream():
            dist.broadcast_object_list(obj_list, src=dist.get_global_rank(self.pg, src)
                                       if self.pg is not dist.group.WORLD else src,
                                       group=self.pg, device=self._device())

    def all_gather_object(self, obj_list: List[Any], obj: Any, frame: int = _FRAME) -> None:
        """``frame``: bytes per rank of the first (usually only) round; small
        payloads (the coalesce gather) pass a smaller one."""
        if self.solo():
            obj_list[0] = obj
            return
        with self._on_side_stream():
            self._all_gather_object(obj_list, obj, max(frame, 64))

    def _all_gather_object(self, obj_list: List[Any], obj: Any, _FRAME: int) -> None:
        ws = self.get_world_size()
        payload = pickle.dumps(obj, protocol=pickle.HIGHEST_PROTOCOL)
        dev = self._device()
        frame = torch.zeros(_FRAME, dtype=torch.uint8)
        head = _HDR.pack(len(payload))
        first = payload[: _FRAME - _HDR.size]
        frame[: _HDR.size] = torch.frombuffer(bytearray(head), dtype=torch.uint8)
        if first:
            frame[_HDR.size: _HDR.size + len(first)] = torch.frombuffer(bytearray(first),
                                                                         dtype=torch.uint8)
        frame = frame.to(dev)
        out = torch.empty(ws * _FRAME, dtype=torch.uint8, device=dev)
        dist.all_gather_into_tensor(out, frame, group=self.pg)
        out = out.cpu().numpy().reshape(ws, _FRAME)
        lens = [_HDR.unpack(out[r, : _HDR.size].tobytes())[0] for r in range(ws)]
        cap = _FRAME - _HDR.size
        over = max(0, max(lens) - cap)
        rest = None
        if over > 0:
            mine = torch.zeros(over, dtype=torch.uint8)
            tail = payload[cap:]
            if tail:
                mine[: len(tail)] = torch.frombuffer(bytearray(tail), dtype=torch.uint8)
            mine = mine.to(dev)
            rest_t = torch.empty(ws * over, dtype=torch.uint8, device=dev)
            dist.all_gather_into_tensor(rest_t, mine, group=self.pg)
            rest = rest_t.cpu().numpy().reshape(ws, over)
        for r in range(ws):
            n = lens[r]
            body = out[r, _HDR.size: _HDR.size + min(n, cap)].tobytes()
            if n > cap:
                body += rest[r, : n - cap].tobytes()
            obj_list[r] = pickle.loads(body)

    def scatter_object_list(self, output_list: List[Any], input_list: Optional[List[Any]],
                            src: int = 0) -> None:
        if self.solo():
            output_list[0] = input_list[0] if input_list else None
            return
        # RCCL has no scatter of objects: broadcast the whole list, keep ours
        # (reference falls back the same way for NCCL, pg_wrapper.py:58-89)
        objs = [input_list] if self.get_rank() == src else [None]
        self.broadcast_object_list(objs, src=src)
        output_list[0] = objs[0][self.get_rank()]


# reference-compatible name
PGWrapper = Comm
