"""RSS sampling around a code region (reference `rss_profiler.py:17-56`)."""

from __future__ import annotations

import threading
import time
from contextlib import contextmanager
from typing import Generator, List

import psutil


@contextmanager
def measure_rss_deltas(rss_deltas: List[int], interval_s: float = 0.1
                       ) -> Generator[None, None, None]:
    """Append (RSS - RSS at entry) every ``interval_s`` to ``rss_deltas``."""
    proc = psutil.Process()
    base = proc.memory_info().rss
    stop = threading.Event()

    def sample() -> None:
        while not stop.is_set():
            rss_deltas.append(proc.memory_info().rss - base)
            stop.wait(interval_s)

    th = threading.Thread(target=sample, daemon=True)
    th.start()
    try:
        yield
    finally:
        stop.set()
        th.join()
        rss_deltas.append(proc.memory_info().rss - base)


def peak_rss_delta(fn, *args, **kwargs):
    deltas: List[int] = []
    t0 = time.monotonic()
    with measure_rss_deltas(deltas):
        out = fn(*args, **kwargs)
    return out, max(deltas) if deltas else 0, time.monotonic() - t0
