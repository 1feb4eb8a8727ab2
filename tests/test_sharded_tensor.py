"""Legacy ``ShardedTensor`` save + resharding across sharding specs.

Mirrors the reference's strategy (tests/test_sharded_tensor_resharding.py:35-108):
several shards all placed on ``rank:0/cpu`` in a 1-rank process group, every
(src spec, dst spec) pair, with and without forced sub-division.
"""

import itertools

import pytest
import torch

from hipsnapshot.utils.test_utils import run_distributed

pytestmark = pytest.mark.multiproc


def _specs():
    from torch.distributed._shard.metadata import ShardMetadata
    from torch.distributed._shard.sharding_spec import ChunkShardingSpec, EnumerableShardingSpec

    return [
        ChunkShardingSpec(dim=0, placements=["rank:0/cpu"] * 4),
        ChunkShardingSpec(dim=1, placements=["rank:0/cpu"] * 3),
        EnumerableShardingSpec([
            ShardMetadata([0, 0], [50, 128], "rank:0/cpu"),
            ShardMetadata([50, 0], [78, 60], "rank:0/cpu"),
            ShardMetadata([50, 60], [78, 68], "rank:0/cpu"),
        ]),
    ]


def _full(st) -> torch.Tensor:
    out = torch.zeros(list(st.metadata().size), dtype=st.dtype)
    for s in st.local_shards():
        o, z = s.metadata.shard_offsets, s.metadata.shard_sizes
        out[o[0]:o[0] + z[0], o[1]:o[1] + z[1]] = s.tensor
    return out


def _worker(tmp: str, subdivide: bool) -> None:
    from torch.distributed._shard import sharded_tensor

    from hipsnapshot import Snapshot, StateDict
    from hipsnapshot.knobs import override_max_shard_size_bytes

    specs = _specs()
    for i, (src, dst) in enumerate(itertools.product(specs, specs)):
        torch.manual_seed(i)
        st = sharded_tensor.rand(src, 128, 128)
        path = f"{tmp}/s{i}"
        if subdivide:
            with override_max_shard_size_bytes(2000):
                Snapshot.take(path, {"sd": StateDict(st=st)})
        else:
            Snapshot.take(path, {"sd": StateDict(st=st)})
        man = Snapshot(path).get_manifest()
        entry = man["0/sd/st"]
        assert entry.type == "ShardedTensor"
        assert all(s.tensor.location.startswith(("sharded/", "batched/")) for s in entry.shards)
        out = sharded_tensor.zeros(dst, 128, 128)
        Snapshot(path).restore({"sd": StateDict(st=out)})
        assert torch.equal(_full(out), _full(st)), (i, subdivide)
        # read_object into a plain tensor
        plain = torch.zeros(128, 128)
        Snapshot(path).read_object("0/sd/st", obj_out=plain)
        assert torch.equal(plain, _full(st))


@pytest.mark.parametrize("subdivide", [False, True])
def test_sharded_tensor_resharding_all_spec_pairs(tmp_path, subdivide):
    run_distributed(_worker, 1, str(tmp_path), subdivide)


def _rank_specs(ws: int):
    """Specs whose shards live on different ranks of a ``ws``-rank group."""
    from torch.distributed._shard.metadata import ShardMetadata
    from torch.distributed._shard.sharding_spec import ChunkShardingSpec, EnumerableShardingSpec

    pl = [f"rank:{r}/cpu" for r in range(ws)]
    return [
        ChunkShardingSpec(dim=0, placements=pl),
        ChunkShardingSpec(dim=1, placements=pl[::-1]),
        EnumerableShardingSpec([
            ShardMetadata([0, 0], [37, 64], pl[0]),
            ShardMetadata([37, 0], [27, 20], pl[1 % ws]),
            ShardMetadata([37, 20], [27, 44], pl[-1]),
        ]),
    ]


def _multirank_worker(tmp: str, subdivide: bool) -> None:
    """Every rank saves its local shards; every (src, dst) spec pair restores
    across ranks; read_object of the whole tensor (with and without a memory
    budget) works on every rank (reference:
    tests/test_sharded_tensor_io_preparer.py:101-175, tests/test_read_object.py:43-140)."""
    import torch.distributed as dist
    from torch.distributed._shard import sharded_tensor

    from hipsnapshot import Snapshot, StateDict
    from hipsnapshot.knobs import override_max_shard_size_bytes
    from hipsnapshot.utils.test_utils import sharded_tensor_eq

    ws = dist.get_world_size()
    specs = _rank_specs(ws)
    for i, (src, dst) in enumerate(itertools.product(specs, specs)):
        torch.manual_seed(i)  # same global values on every rank
        full = torch.randn(64, 64)
        st = sharded_tensor.zeros(src, 64, 64)
        for s in st.local_shards():
            o, z = s.metadata.shard_offsets, s.metadata.shard_sizes
            s.tensor.copy_(full[o[0]:o[0] + z[0], o[1]:o[1] + z[1]])
        path = f"{tmp}/m{i}"
        if subdivide:
            with override_max_shard_size_bytes(1024):
                Snapshot.take(path, {"sd": StateDict(st=st)})
        else:
            Snapshot.take(path, {"sd": StateDict(st=st)})
        out = sharded_tensor.zeros(dst, 64, 64)
        Snapshot(path).restore({"sd": StateDict(st=out)})
        for s in out.local_shards():
            o, z = s.metadata.shard_offsets, s.metadata.shard_sizes
            assert torch.equal(s.tensor, full[o[0]:o[0] + z[0], o[1]:o[1] + z[1]]), (i, o)
        if src is dst:
            assert sharded_tensor_eq(out, st)
        for budget in (None, 4096):
            plain = torch.zeros(64, 64)
            Snapshot(path).read_object("0/sd/st", obj_out=plain, memory_budget_bytes=budget)
            assert torch.equal(plain, full), (i, budget)


@pytest.mark.parametrize("subdivide", [False, True])
def test_sharded_tensor_multirank_resharding(tmp_path, subdivide):
    run_distributed(_multirank_worker, 3, str(tmp_path), subdivide)


def test_subdivide_shard_math():
    from hipsnapshot.io.sharded import ShardedTensorIOPreparer

    t = torch.randn(10, 7)
    pieces = ShardedTensorIOPreparer.subdivide_shard(t, [20, 0], [10, 7], 0, 7 * 4 * 3)
    assert [p[1][0] for p in pieces] == [20, 23, 26, 29]
    assert [p[2][0] for p in pieces] == [3, 3, 3, 1]
    assert torch.equal(torch.cat([p[0] for p in pieces]), t)
    pieces = ShardedTensorIOPreparer.subdivide_shard(t, [0, 5], [10, 7], 1, 10 * 4 * 2)
    assert [p[2][1] for p in pieces] == [2, 2, 2, 1]
    # a slice larger than the limit still yields 1-row pieces
    pieces = ShardedTensorIOPreparer.subdivide_shard(t, [0, 0], [10, 7], 0, 1)
    assert len(pieces) == 10
    with pytest.raises(ValueError):
        ShardedTensorIOPreparer.subdivide_shard(t, [0, 0], [10, 7], 0, 0)


def test_overlap_math():
    from hipsnapshot.io.sharded import overlap_narrows

    assert overlap_narrows([0, 0], [10, 10], [5, 5], [10, 10]) == [(0, 5, 0, 5), (1, 5, 0, 5)]
    assert overlap_narrows([0, 0], [10, 10], [10, 0], [5, 5]) is None
    assert overlap_narrows([4], [4], [0], [6]) == [(0, 0, 4, 2)]
