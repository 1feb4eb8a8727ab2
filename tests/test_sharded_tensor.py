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
