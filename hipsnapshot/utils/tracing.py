"""Observability: roctx ranges, a periodic write-progress reporter, JSON timing records.

* ``roctx_range(name)`` -- pushes a ROCTx range (``libroctx64.so`` from the torch
  ROCm wheel or ``/opt/rocm``) so ``rocprofv3 --marker-trace`` shows
  stage / D2H / write / commit phases next to the HIP kernels.  Enabled with
  ``HIPSNAPSHOT_ROCTX=1``; a no-op otherwise.
* ``WriteReporter`` -- the reference's ``_WriteReporter``
  (`/root/reference/torchsnapshot/scheduler.py:93-175`): a DEBUG-level table of
  per-rank progress (staged / written / in-flight bytes, RSS delta, budget)
  logged every ``interval_s`` while a write pipeline runs.
"""

from __future__ import annotations

import contextlib
import ctypes
import glob
import logging
import os
import time
from typing import Optional

import psutil

logger = logging.getLogger("hipsnapshot.scheduler")

_roctx = None
_roctx_tried = False


def _load_roctx():
    global _roctx, _roctx_tried
    if _roctx_tried:
        return _roctx
    _roctx_tried = True
    if os.environ.get("HIPSNAPSHOT_ROCTX", "0") != "1":
        return None
    cands = []
    try:
        import torch

        cands += glob.glob(os.path.join(os.path.dirname(torch.__file__), "lib", "libroctx64.so*"))
    except Exception:  # pragma: no cover
        pass
    cands += glob.glob("/opt/rocm/lib/libroctx64.so*")
    for c in cands:
        try:
            lib = ctypes.CDLL(c)
            lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
            lib.roctxRangePushA.restype = ctypes.c_int
            lib.roctxRangePop.restype = ctypes.c_int
            _roctx = lib
            break
        except OSError:
            continue
    return _roctx


@contextlib.contextmanager
def roctx_range(name: str):
    lib = _load_roctx()
    if lib is None:
        yield
        return
    lib.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        lib.roctxRangePop()


class WriteReporter:
    def __init__(self, rank: int, memory_budget_bytes: int, interval_s: float = 5.0) -> None:
        self.rank = rank
        self.budget = memory_budget_bytes
        self.interval_s = interval_s
        self.t0 = time.monotonic()
        self.last = self.t0
        self.rss0 = psutil.Process().memory_info().rss

    def maybe_report(self, n_pending: int, n_staging: int, n_io: int, in_use: int,
                     bytes_written: int, force: bool = False) -> Optional[str]:
        now = time.monotonic()
        if not force and now - self.last < self.interval_s:
            return None
        if not logger.isEnabledFor(logging.DEBUG) and not force:
            return None
        self.last = now
        rss = psutil.Process().memory_info().rss - self.rss0
        line = (f"rank {self.rank} t={now - self.t0:7.2f}s stage-able={n_pending:5d} "
                f"staging={n_staging:3d} writing={n_io:4d} in-use={in_use / 2**30:7.2f}GiB "
                f"rss-delta={rss / 2**30:7.2f}GiB budget={self.budget / 2**30:7.2f}GiB "
                f"written={bytes_written / 1e9:8.3f}GB")
        logger.debug(line)
        return line
