"""Randomised distributed round trips (4 gloo ranks on the CPU): random
DTensor layouts -- 1-D and 2-D meshes, ``Shard`` / ``Replicate`` on any dim,
uneven shapes -- saved, then restored into ANOTHER random layout (elastic
resharding, HSDP replica splits, replicated <-> sharded) and read whole with
``read_object``; every case is compared with the global tensor.  torch's own
``distribute_tensor`` builds both layouts, so the ground truth is not ours.

Reference: the hand-picked resharding matrix of
`/root/reference/tests/test_sharded_tensor_resharding.py`.
"""

import os
import random

import pytest
import torch

from hipsnapshot.utils.test_utils import run_distributed

pytestmark = pytest.mark.multiproc

MESHES = [(4,), (2, 2), (1, 4), (4, 1)]


def _layout(rng: random.Random, ndim: int, strided: bool = False):
    from torch.distributed.tensor import Replicate, Shard
    from torch.distributed.tensor.placement_types import _StridedShard

    mesh = rng.choice(MESHES)
    pl = []
    for _ in mesh:
        r = rng.random()
        if strided and r < 0.3:
            pl.append(_StridedShard(rng.randrange(ndim), split_factor=rng.randint(2, 3)))
        elif r < 0.75:
            pl.append(Shard(rng.randrange(ndim)))
        else:
            pl.append(Replicate())
    return mesh, pl


def _truth_index(shape, mesh_shape, coord, placements):
    """Global indices per dim of a coordinate's local tensor, by torch's own
    splitting code (``_split_tensor``): the ground truth, not ours."""
    from torch.distributed.tensor import Shard
    from torch.distributed.tensor.placement_types import _StridedShard

    idx = [torch.arange(n) for n in shape]
    for mdim, p in enumerate(placements):
        if not hasattr(p, "dim"):
            continue
        p1 = _StridedShard(0, split_factor=p.split_factor) if isinstance(p, _StridedShard) \
            else Shard(0)
        shards, _ = p1._split_tensor(idx[p.dim], mesh_shape[mdim], with_padding=False)
        idx[p.dim] = shards[coord[mdim]]
    return idx


def _worker(root: str, n_cases: int, seed: int, device: str = "cpu",
            strided: bool = False) -> None:
    import torch.distributed as dist
    from torch.distributed.device_mesh import init_device_mesh
    from torch.distributed.tensor import DTensor, distribute_tensor

    from hipsnapshot import Snapshot, StateDict, knobs

    rng = random.Random(seed)  # the same stream on every rank
    meshes = {}
    if device.startswith("cuda"):  # before any "cuda" mesh picks rank % n_gpus
        torch.cuda.set_device(torch.device(device))

    def mesh_of(shape, dev_type="cpu"):
        if (shape, dev_type) not in meshes:
            meshes[(shape, dev_type)] = init_device_mesh(dev_type, shape)
        return meshes[(shape, dev_type)]

    def place(glob, shape, pl):
        """``glob`` laid out by torch (on a CPU mesh), then, for a GPU run,
        the same local pieces as DTensors of HIP tensors (no collectives on
        them: gloo ranks share the one GPU).  Layouts with a _StridedShard
        (FSDP2 over TP) are cut by torch's ``_split_tensor``."""
        if any(type(p).__name__ == "_StridedShard" for p in pl):
            mesh = mesh_of(shape, "cuda" if device != "cpu" else "cpu")
            coord = mesh.get_coordinate()
            local = glob[torch.meshgrid(*_truth_index(list(glob.shape), shape, coord, pl),
                                        indexing="ij")].contiguous()
            return DTensor.from_local(local.to(device), mesh, pl, run_check=False,
                                      shape=glob.shape, stride=glob.stride())
        cpu = distribute_tensor(glob, mesh_of(shape), pl)
        if device == "cpu":
            return cpu
        return DTensor.from_local(cpu.to_local().to(device), mesh_of(shape, "cuda"), pl,
                                  run_check=False, shape=cpu.shape, stride=cpu.stride())

    for case in range(n_cases):
        ndim = rng.randint(1, 3)
        shape = [rng.randint(1, 13) for _ in range(ndim)]
        dtype = rng.choice([torch.float32, torch.bfloat16, torch.int64, torch.float64])
        g = torch.Generator().manual_seed(seed * 1000 + case)
        glob = (torch.randn(shape, generator=g) * 100).to(dtype)
        save_mesh, save_pl = _layout(rng, ndim, strided)
        load_mesh, load_pl = _layout(rng, ndim, strided)
        compression = rng.choice(["none", "hsz1", "hsz1+host"])
        batching = rng.random() < 0.7
        use_async = rng.random() < 0.4
        what = (case, shape, dtype, save_mesh, save_pl, load_mesh, load_pl, compression,
                batching, use_async)
        path = os.path.join(root, f"c{case}")
        src = place(glob, save_mesh, save_pl)
        with knobs.override_is_batching_disabled(not batching):
            app = {"s": StateDict(t=src, step=case)}
            if use_async:
                snap = Snapshot.async_take(path, app, compression=compression).wait()
            else:
                snap = Snapshot.take(path, app, compression=compression)
            # a DTensor target of another float dtype is cast in place
            tdt = rng.choice([torch.float32, torch.bfloat16, torch.float64]) \
                if dtype.is_floating_point and rng.random() < 0.3 else dtype
            dst = place(torch.zeros(glob.shape, dtype=tdt), load_mesh, load_pl)
            app = {"s": StateDict(t=dst, step=-1)}
            Snapshot(path).restore(app)
        got = app["s"]["t"].to_local().cpu()
        want = place(glob.to(tdt), load_mesh, load_pl).to_local().cpu()
        assert got.dtype == tdt and torch.equal(got, want), (what, tdt)
        assert app["s"]["step"] == case, what
        whole = torch.zeros_like(glob, device=device)
        snap.read_object("0/s/t", obj_out=whole)
        assert torch.equal(whole.cpu(), glob), what
        dist.barrier()


@pytest.mark.slow  # the strided test below covers plain placements too (CPU time)
@pytest.mark.parametrize("seed", [1])
def test_random_dtensor_layouts_reshard_exactly(tmp_path, seed):
    run_distributed(_worker, 4, str(tmp_path), 10, seed, timeout=400)


def test_random_strided_dtensor_layouts_reshard_exactly(tmp_path):
    """The same with _StridedShard placements (FSDP2 over TP) mixed in: a
    local tensor holds several disjoint runs of a dim."""
    run_distributed(_worker, 4, str(tmp_path), 8, 3, "cpu", True, timeout=400)


@pytest.mark.gpu
def test_random_dtensor_layouts_reshard_exactly_gpu(gpu, tmp_path):
    """The same with every local piece on cuda:0 (4 gloo ranks sharing it):
    staging, HSZ1 and the native restore's scatter under random layouts."""
    run_distributed(_worker, 4, str(tmp_path), 24, 7, "cuda:0", timeout=600)


def _elastic_state(seed: int, world: int):
    """Replicated tensors (the same on every rank; large ones chunked and
    spread by the partitioner) and a Shard(0) DTensor over the world."""
    import torch.distributed as dist  # noqa: F401
    from torch.distributed.device_mesh import init_device_mesh
    from torch.distributed.tensor import Shard, distribute_tensor

    rng = random.Random(seed)
    g = torch.Generator().manual_seed(seed)
    rep = {f"r{i}": (torch.randn(rng.choice([3, 1000, 70_000]), generator=g) * 10).to(
        rng.choice([torch.float32, torch.bfloat16])) for i in range(rng.randint(1, 6))}
    rows = rng.randint(1, 40)
    glob = torch.randn(rows, rng.randint(1, 9), generator=g)
    mesh = init_device_mesh("cpu", (world,))
    return rep, glob, distribute_tensor(glob, mesh, [Shard(0)])


def _elastic_save(root: str, seed: int) -> None:
    import torch.distributed as dist

    from hipsnapshot import Snapshot, StateDict, knobs

    rep, _glob, dt = _elastic_state(seed, dist.get_world_size())
    with knobs.override_max_chunk_size_bytes(64 << 10):
        Snapshot.take(root, {"rep": StateDict(**rep), "sh": StateDict(w=dt)},
                      replicated=["rep/**"],
                      compression=random.Random(seed).choice(["none", "hsz1+host"]))


def _elastic_restore(root: str, seed: int) -> None:
    import torch.distributed as dist

    from hipsnapshot import Snapshot, StateDict

    rep, glob, dt = _elastic_state(seed, dist.get_world_size())
    out_rep = StateDict(**{k: torch.zeros_like(v) for k, v in rep.items()})
    dt.to_local().zero_()
    out_sh = StateDict(w=dt)
    Snapshot(root).restore({"rep": out_rep, "sh": out_sh})
    for k, v in rep.items():
        assert torch.equal(out_rep[k], v), (seed, k)
    assert torch.equal(out_sh["w"].full_tensor(), glob), seed


@pytest.mark.slow  # 10 s of spawned ranks; --run-slow (CI) runs it
@pytest.mark.parametrize("seed", range(11, 11 + int(os.environ.get("HS_ELASTIC_SEEDS", "1"))))
def test_random_elastic_world_sizes(tmp_path, seed):
    """Save with W1 ranks, restore with W2 (random in 1-4): replicated state
    partitioned over the savers comes back whole on every restoring rank, a
    Shard(0) DTensor re-cut for W2."""
    rng = random.Random(seed)
    for i in range(1):
        w1, w2 = rng.randint(1, 4), rng.randint(1, 4)
        path = str(tmp_path / f"e{i}")
        run_distributed(_elastic_save, w1, path, seed * 10 + i, timeout=240)
        run_distributed(_elastic_restore, w2, path, seed * 10 + i, timeout=240)


def _random_spec(rng: random.Random, shape, world: int):
    """A random ChunkShardingSpec or a random grid EnumerableShardingSpec of a
    2-D tensor, shards on random ranks."""
    from torch.distributed._shard.metadata import ShardMetadata
    from torch.distributed._shard.sharding_spec import ChunkShardingSpec, EnumerableShardingSpec

    if rng.random() < 0.5:
        k = rng.randint(1, 5)
        return ChunkShardingSpec(dim=rng.randrange(2),
                                 placements=[f"rank:{rng.randrange(world)}/cpu" for _ in range(k)])
    cuts = []
    for n in shape:
        c = sorted(set(rng.sample(range(1, n), min(n - 1, rng.randint(0, 3))))) if n > 1 else []
        cuts.append([0] + c + [n])
    shards = [ShardMetadata([r0, c0], [r1 - r0, c1 - c0], f"rank:{rng.randrange(world)}/cpu")
              for r0, r1 in zip(cuts[0], cuts[0][1:]) for c0, c1 in zip(cuts[1], cuts[1][1:])]
    return EnumerableShardingSpec(shards)


def _sharded_worker(root: str, n_cases: int, seed: int) -> None:
    import torch.distributed as dist
    from torch.distributed._shard import sharded_tensor

    from hipsnapshot import Snapshot, StateDict
    from hipsnapshot.knobs import override_max_shard_size_bytes

    world = dist.get_world_size()
    rng = random.Random(seed)

    def make(spec, glob):
        st = sharded_tensor.empty(spec, *glob.shape, dtype=glob.dtype)
        for s in st.local_shards():
            o, z = s.metadata.shard_offsets, s.metadata.shard_sizes
            s.tensor.copy_(glob[o[0]:o[0] + z[0], o[1]:o[1] + z[1]])
        return st

    for case in range(n_cases):
        shape = [rng.randint(1, 30), rng.randint(1, 30)]
        g = torch.Generator().manual_seed(seed * 100 + case)
        glob = torch.randn(shape, generator=g)
        src_spec, dst_spec = _random_spec(rng, shape, world), _random_spec(rng, shape, world)
        sub = rng.choice([None, 64, 400])
        path = os.path.join(root, f"st{case}")
        src = make(src_spec, glob)
        if sub:
            with override_max_shard_size_bytes(sub):
                Snapshot.take(path, {"sd": StateDict(st=src)})
        else:
            Snapshot.take(path, {"sd": StateDict(st=src)})
        dst = make(dst_spec, torch.zeros_like(glob))
        Snapshot(path).restore({"sd": StateDict(st=dst)})
        for s in dst.local_shards():
            o, z = s.metadata.shard_offsets, s.metadata.shard_sizes
            assert torch.equal(s.tensor, glob[o[0]:o[0] + z[0], o[1]:o[1] + z[1]]), \
                (case, shape, src_spec, dst_spec, sub)
        whole = torch.zeros_like(glob)
        Snapshot(path).read_object("0/sd/st", obj_out=whole)
        assert torch.equal(whole, glob), (case, "read_object")
        dist.barrier()


@pytest.mark.parametrize("world", [3])
def test_random_sharded_tensor_specs_reshard_exactly(tmp_path, world):
    """Legacy ShardedTensor: random Chunk / Enumerable (grid) specs on random
    ranks, saved (with and without forced sub-division) and restored into
    another random spec, then read whole.  The reference's own test crosses 3
    fixed specs (`/root/reference/tests/test_sharded_tensor_resharding.py`)."""
    run_distributed(_sharded_worker, world, str(tmp_path), 10,
                    int(os.environ.get("HS_ST_SEED", "5")) + world, timeout=400)


def _comm_worker(n_rounds: int, seed: int) -> None:
    """Comm's framed all-gather / broadcast / scatter with random payload
    sizes per rank (0 B to ~3 frames, the frame size itself random): every
    take's metadata exchange rides on them."""
    import torch.distributed as dist

    from hipsnapshot.parallel.comm import Comm

    comm = Comm()
    rank, ws = comm.get_rank(), comm.get_world_size()
    rng = random.Random(seed)  # the same draws on every rank
    for i in range(n_rounds):
        frame = rng.choice([64, 1000, 1 << 16])
        sizes = [rng.choice([0, 1, frame - 1, frame, frame + 1, rng.randint(0, 3 * frame)])
                 for _ in range(ws)]
        payload = {"r": rank, "i": i, "b": bytes([rank % 256]) * sizes[rank]}
        out = [None] * ws
        comm.all_gather_object(out, payload, frame=frame)
        for r in range(ws):
            assert out[r] == {"r": r, "i": i, "b": bytes([r % 256]) * sizes[r]}, (i, r, frame)
        src = rng.randrange(ws)
        obj = [("from", rank, "x" * sizes[rank])]
        comm.broadcast_object_list(obj, src=src)
        assert obj == [("from", src, "x" * sizes[src])], (i, "broadcast")
        res = [None]
        comm.scatter_object_list(res, [(r, "y" * sizes[r]) for r in range(ws)]
                                 if rank == src else None, src=src)
        assert res[0] == (rank, "y" * sizes[rank]), (i, "scatter")
    dist.barrier()


@pytest.mark.slow  # 4 s of spawned ranks; --run-slow (CI) runs it
@pytest.mark.parametrize("world", [3])
def test_random_comm_payloads(world):
    run_distributed(_comm_worker, world, 40, 17 + world, timeout=240)


@pytest.mark.gpu
def test_random_comm_payloads_rccl_forced(gpu, monkeypatch):
    """The same payloads over a one-rank RCCL group with
    HIPSNAPSHOT_FORCE_COLLECTIVES (device-tensor frames, overflow rounds)."""
    monkeypatch.setenv("HIPSNAPSHOT_FORCE_COLLECTIVES", "1")
    run_distributed(_comm_worker, 1, 40, 23, backend="nccl", timeout=240)
