"""Key-value store bootstrap and the two-phase commit barrier.

Reference: `/root/reference/torchsnapshot/dist_store.py:17-196`.  The async
commit thread must not issue collectives (they could interleave with the
trainer's RCCL calls), so ranks synchronise through c10d ``Store`` keys:

* ``get_or_create_store`` reuses the default c10d store, or bootstraps a
  ``TCPStore`` (rank 0 picks a free port on 127.0.0.1-reachable host and
  broadcasts it) when the job has none;
* ``LinearBarrier`` = arrive (peers -> leader) / depart (leader -> peers)
  with error propagation through the keys.  Keys carry a per-snapshot nonce so
  two snapshots to the same path never see each other's stale keys (the
  reference keyed by path only), and ``depart`` marks the barrier departed
  (reference set ``arrived`` again, Appendix C #5).
* A barrier leaves no keys behind: the leader deletes the peers' keys once it
  has read them in ``arrive``, and the last peer to read the leader's key in
  ``depart`` deletes it (a counter key says which peer is last).  Every
  ``async_take`` of a long job used to add ~2 x world size keys to the default
  c10d store for good.  Keys of a barrier that failed are left (they carry
  the error).
"""

from __future__ import annotations

import socket
from datetime import timedelta
from typing import Dict, Optional

import torch.distributed as dist

from .comm import Comm

DEFAULT_TCP_STORE_TIMEOUT = timedelta(seconds=600)
_pg_to_store: Dict[object, dist.Store] = {}


def existing_store(comm: Comm) -> Optional[dist.Store]:
    """The default c10d store, or one ``create_store`` made earlier for this
    group; None if neither exists.  Never issues a collective."""
    if dist.is_initialized():
        try:
            store = dist.distributed_c10d._get_default_store()
        except Exception:  # pragma: no cover - MPI backend
            store = None
        if store is not None:
            return store
    return _pg_to_store.get(comm.pg)


def get_or_create_store(comm: Comm) -> dist.Store:
    store = existing_store(comm)
    if store is not None:
        return store
    return create_store(comm)


def _free_port(host: str) -> int:
    s = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
    s.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
    s.bind((host, 0))
    port = s.getsockname()[1]
    s.close()
    return port


def create_store(comm: Comm, host: Optional[str] = None) -> dist.Store:
    if comm.get_rank() == 0:
        if host is None:
            try:
                host = socket.gethostbyname(socket.gethostname())
            except OSError:
                host = "127.0.0.1"
            if comm.get_world_size() == 1:
                host = "127.0.0.1"
        obj = [host, _free_port(host if host != "0.0.0.0" else "127.0.0.1")]
    else:
        obj = [None, None]
    comm.broadcast_object_list(obj, src=0)
    store = dist.TCPStore(host_name=obj[0], port=obj[1], world_size=comm.get_world_size(),
                          is_master=comm.get_rank() == 0, timeout=DEFAULT_TCP_STORE_TIMEOUT,
                          wait_for_workers=True)
    _pg_to_store[comm.pg] = store
    return store


class LinearBarrier:
    """Two-phase barrier; the leader acts between ``arrive`` and ``depart``.

    ``report_error`` (any rank, before its next phase) makes the leader raise
    in ``arrive`` and every peer raise in ``depart``.
    """

    def __init__(self, prefix: str, store: dist.Store, rank: int, world_size: int,
                 leader_rank: int = 0) -> None:
        self.prefix = prefix
        self.store = store
        self.rank = rank
        self.world_size = world_size
        self.leader_rank = leader_rank
        self.arrived = False
        self.departed = False
        self._errored = False

    def _key(self, rank: int) -> str:
        return f"{self.prefix}_{rank}"

    def _delete(self, keys) -> None:
        for k in keys:
            try:
                self.store.delete_key(k)
            except Exception:  # noqa: BLE001 - a store without delete: keys stay
                return

    def arrive(self, timeout: timedelta) -> None:
        if self.arrived:
            raise RuntimeError("Can't call .arrive() multiple times on a barrier.")
        if self.departed:
            raise RuntimeError("Can't call .arrive() on a completed barrier.")
        self.arrived = True
        if self.rank != self.leader_rank:
            if not self._errored:  # never overwrite a reported error
                self.store.set(self._key(self.rank), "")
            return
        peers = [self._key(r) for r in range(self.world_size) if r != self.leader_rank]
        if peers:
            self.store.wait(peers, timeout)
        for k in peers:
            err = self.store.get(k)
            if len(err) != 0:
                msg = err.decode() if isinstance(err, bytes) else str(err)
                self.report_error(msg)
                raise RuntimeError(msg)
        self._delete(peers)

    def depart(self, timeout: timedelta) -> None:
        if not self.arrived:
            raise RuntimeError("Can't call .depart() before calling .arrive() on a barrier.")
        if self.departed:
            raise RuntimeError("Can't call .depart() on a completed barrier.")
        self.departed = True
        if self.rank == self.leader_rank:
            self.store.set(self._key(self.leader_rank), "")
            return
        lk = self._key(self.leader_rank)
        self.store.wait([lk], timeout)
        err = self.store.get(lk)
        if len(err) != 0:
            raise RuntimeError(err.decode() if isinstance(err, bytes) else str(err))
        done = f"{self.prefix}_departed"
        if self.store.add(done, 1) == self.world_size - 1:  # the last peer out
            self._delete([lk, done])

    def report_error(self, err: str) -> None:
        self._errored = True
        self.store.set(self._key(self.rank), f"Rank {self.rank} encountered error: {err}")
