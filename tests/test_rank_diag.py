"""utils/rank_diag.py: the per-rank phase split bench.py prints for N > 1,
on 2 gloo ranks (CPU tensors)."""

import pytest
import torch

from hipsnapshot.utils import rank_diag
from hipsnapshot.utils.test_utils import run_distributed


def _worker(tmp):
    import torch.distributed as dist

    from hipsnapshot import Snapshot, StateDict

    sd = StateDict(**{f"w{i}": torch.randn(256, 1024) for i in range(4)})
    d = rank_diag.measure(lambda: Snapshot.take(f"{tmp}/s", {"sd": sd}))
    assert d["take_ms"] > 0 and d["cpu_s"] >= 0
    assert d["write_bytes"] >= 4 * 256 * 1024 * 4  # this rank's blobs
    assert d["page_cache_GBps"] and d["write_busy_s"] > 0
    assert d["meta_total_ms"] > 0 and "gather_manifest" in d["meta_ms"], d["meta_ms"]
    assert d["cpu_set"]["n"] >= 1
    allr = [None] * dist.get_world_size()
    dist.all_gather_object(allr, d)
    sk = rank_diag.skew(allr)
    assert sk["take_ms_max_over_median"] >= 1.0
    assert sk["slowest_rank"] in (0, 1)
    assert sk["slowest_rank_phase"] in ("d2h_busy_s", "write_busy_s", "meta_critical_ms")
    assert d["meta_critical_ms"] <= d["meta_total_ms"]


@pytest.mark.multiproc
def test_rank_diag_two_ranks(tmp_path):
    run_distributed(_worker, 2, str(tmp_path))


def test_union_and_cpu_set():
    ev = [{"ts": 0, "dur": 10}, {"ts": 5, "dur": 10}, {"ts": 30, "dur": 5}]
    assert rank_diag._union_s(ev) == pytest.approx(20e-6)
    assert rank_diag.cpu_set()["n"] >= 1
