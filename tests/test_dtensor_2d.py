"""2-D DTensor layouts: FSDP2 over tensor parallel (``_StridedShard``),
HSDP, multi-dim meshes, and resharding between them.

The reference reshards arbitrary ShardedTensor layouts
(`/root/reference/torchsnapshot/io_preparers/sharded_tensor.py:127-170, 195-268`,
tests `tests/test_sharded_tensor_resharding.py:35-108`).  torch 2.10's
``fully_shard`` over a ``parallelize_module`` model produces
``(_StridedShard(0, sf=tp), Shard(0))`` placements; these tests save such a
model (+ AdamW state) on a (dp=2, tp=2) mesh and restore it bitwise into a
(tp=2, dp=2) mesh (every rank's coordinates change), a 1-D FSDP (4,) mesh
and a single unsharded process, plus ``read_object`` into plain tensors.
"""

import itertools
import random

import pytest
import torch

from hipsnapshot.utils.test_utils import run_distributed


def _cfg():
    from hipsnapshot.models.llama import LlamaConfig

    cfg = LlamaConfig.tiny()
    cfg.vocab_size, cfg.ffn_dim = 509, 250  # uneven splits on every mesh
    return cfg


# ---------------------------------------------------------------------------
# layout math (no process group)


def _truth(gshape, mesh_shape, coord, placements):
    """Global indices per dim by torch's own splitting code (ground truth)."""
    from torch.distributed.tensor import Shard
    from torch.distributed.tensor.placement_types import _StridedShard

    idx = [torch.arange(n) for n in gshape]
    for mdim, p in enumerate(placements):
        if not hasattr(p, "dim"):
            continue
        d = p.dim
        p1 = _StridedShard(0, split_factor=p.split_factor) if isinstance(p, _StridedShard) \
            else Shard(0)  # split the 1-D index list of dim d
        shards, _ = p1._split_tensor(idx[d], mesh_shape[mdim], with_padding=False)
        idx[d] = shards[coord[mdim]]
    return [t.tolist() for t in idx]


def _expand(runs):
    return [[g + i for g, ln in dr for i in range(ln)] for dr in runs]


def test_dim_index_runs_docstring_example():
    from torch.distributed.tensor import Shard
    from torch.distributed.tensor.placement_types import _StridedShard

    from hipsnapshot.io.sharded import dim_index_runs

    pl = [Shard(0), _StridedShard(0, split_factor=2)]
    got = {c: _expand(dim_index_runs([8], [2, 2], c, pl))[0]
           for c in itertools.product(range(2), range(2))}
    assert got == {(0, 0): [0, 2], (0, 1): [1, 3], (1, 0): [4, 6], (1, 1): [5, 7]}
    # FSDP2 x TP order: right-to-left sharding, contiguous per rank
    pl = [_StridedShard(0, split_factor=2), Shard(0)]
    got = {c: dim_index_runs([8], [2, 2], c, pl)[0] for c in itertools.product(range(2), range(2))}
    assert got == {(0, 0): [(0, 2)], (0, 1): [(4, 2)], (1, 0): [(2, 2)], (1, 1): [(6, 2)]}


def test_dim_index_runs_matches_torch_random():
    from torch.distributed.tensor import Replicate, Shard
    from torch.distributed.tensor.placement_types import _StridedShard

    from hipsnapshot.io.sharded import dim_index_runs, runs_to_boxes

    rng = random.Random(0)
    for _ in range(400):
        nd = rng.randint(1, 3)
        gshape = [rng.randint(1, 23) for _ in range(nd)]
        mdims = rng.randint(1, 3)
        mesh = [rng.randint(1, 4) for _ in range(mdims)]
        pl = []
        for _m in range(mdims):
            k = rng.random()
            d = rng.randrange(nd)
            if k < 0.2:
                pl.append(Replicate())
            elif k < 0.6:
                pl.append(Shard(d))
            else:
                pl.append(_StridedShard(d, split_factor=rng.randint(1, 4)))
        for coord in itertools.product(*[range(m) for m in mesh]):
            truth = _truth(gshape, mesh, coord, pl)
            runs = dim_index_runs(gshape, mesh, coord, pl)
            assert _expand(runs) == truth, (gshape, mesh, pl, coord)
            # boxes tile the local tensor exactly
            boxes = runs_to_boxes(runs)
            vol = sum(int(torch.tensor(sz).prod()) for _lo, _go, sz in boxes)
            assert vol == int(torch.tensor([len(t) for t in truth]).prod())


# ---------------------------------------------------------------------------
# multi-rank save / restore


def _mesh2d(order, device="cpu"):
    from torch.distributed.device_mesh import init_device_mesh

    if torch.device(device).type == "cuda":  # all ranks share this GPU
        torch.cuda.set_device(torch.device(device))
    return init_device_mesh(torch.device(device).type, (2, 2), mesh_dim_names=order)


def _with_adamw(model):
    opt = torch.optim.AdamW(model.parameters(), lr=1e-3, foreach=False)
    for p in model.parameters():
        p.grad = torch.zeros_like(p)
    opt.step()
    opt.zero_grad(set_to_none=True)
    return opt


def _full(v):
    if not hasattr(v, "full_tensor"):
        return v
    if not v.is_cuda:
        return v.full_tensor()
    # HIP tensors: a 1-D mesh over the whole world gets a "cuda:nccl" group
    # from DeviceMesh even under a gloo default group, and RCCL refuses
    # several ranks on one GPU -- assemble the full tensor from every rank's
    # local boxes over the (gloo) default group instead.  (On the CPU the
    # same boxes are checked against full_tensor() in _save_worker.)
    import torch.distributed as dist

    from hipsnapshot.io.sharded import local_boxes

    mine = [(b.offsets, b.sizes, b.tensor.cpu()) for b in local_boxes(v)]
    every = [None] * dist.get_world_size()
    dist.all_gather_object(every, mine)
    out = torch.zeros(tuple(v.shape), dtype=v.dtype)
    for boxes in every:
        for o, sz, t in boxes:
            out[tuple(slice(a, a + n) for a, n in zip(o, sz))] = t
    return out


def _flat_state(model, opt):
    out = {f"m/{k}": _full(v).cpu().clone() for k, v in model.state_dict().items()}
    for i, st in opt.state_dict()["state"].items():
        for k, v in st.items():
            if torch.is_tensor(v) and v.dim() > 0:
                out[f"o/{i}/{k}"] = _full(v).cpu().clone()
    return out


def _zero_(model, opt):
    for p in model.parameters():
        (p._local_tensor if hasattr(p, "_local_tensor") else p.data).zero_()
    for st in opt.state.values():
        for k, v in st.items():
            if torch.is_tensor(v) and v.dim() > 0:
                (v._local_tensor if hasattr(v, "_local_tensor") else v).zero_()


def _save_worker(tmp: str, device: str = "cpu"):
    import torch.distributed as dist

    from hipsnapshot import Snapshot
    from hipsnapshot.io.sharded import local_boxes
    from hipsnapshot.knobs import override_max_shard_size_bytes
    from hipsnapshot.models.llama import build_2d_llama

    model = build_2d_llama(_cfg(), torch.device(device), _mesh2d(("dp", "tp"), device),
                           torch.float32)
    opt = _with_adamw(model)
    with torch.no_grad():
        # globally consistent moments (TP replicas of a norm's state agree)
        gen = torch.Generator().manual_seed(100)
        for st in opt.state.values():
            for k in ("exp_avg", "exp_avg_sq"):
                full = torch.rand(st[k].shape, generator=gen).to(device)
                for b in local_boxes(st[k]):
                    b.tensor.copy_(full[tuple(slice(o, o + s)
                                              for o, s in zip(b.offsets, b.sizes))])
    kinds = {type(p).__name__ for v in model.state_dict().values() for p in v.placements}
    assert "_StridedShard" in kinds, kinds
    # every box the write path sees is where full_tensor() says it is
    for k, v in model.state_dict().items():
        full = _full(v).to(v.device) if v.is_cuda else v.full_tensor()
        for b in local_boxes(v, for_write=True):
            sl = tuple(slice(o, o + s) for o, s in zip(b.offsets, b.sizes))
            assert torch.equal(full[sl], b.tensor), k
    ref = _flat_state(model, opt)
    app = {"model": model, "optim": opt}
    Snapshot.take(f"{tmp}/sync", app)
    man = Snapshot(f"{tmp}/sync").get_manifest()
    norm = [s.offsets for k, e in man.items() if k.endswith("/model/norm.weight")
            for s in e.shards]
    assert sorted(norm) == [[0], [64]], norm  # TP replicas of the dp-sharded norm write once
    with override_max_shard_size_bytes(4096):  # forced sub-division of every box
        Snapshot.async_take(f"{tmp}/async", app).wait()
    if dist.get_rank() == 0:
        torch.save(ref, f"{tmp}/ref.pt")


def _check(model, opt, ref, tag):
    got = _flat_state(model, opt)
    assert got.keys() == ref.keys(), tag
    for k in ref:
        assert torch.equal(got[k], ref[k]), (tag, k)


def _restore_worker(tmp: str, target: str, device: str = "cpu"):
    import torch.distributed as dist
    from torch.distributed.device_mesh import init_device_mesh

    from hipsnapshot import Snapshot
    from hipsnapshot.models.llama import Llama, build_2d_llama, build_fsdp_llama

    ref = torch.load(f"{tmp}/ref.pt", weights_only=True)
    dev = torch.device(device)
    if target == "2d_swapped":
        model = build_2d_llama(_cfg(), dev, _mesh2d(("tp", "dp"), device), torch.float32)
    elif target == "2d_same":
        model = build_2d_llama(_cfg(), dev, _mesh2d(("dp", "tp"), device), torch.float32)
    elif target == "fsdp":
        if dev.type == "cuda":
            torch.cuda.set_device(dev)
        mesh = init_device_mesh(dev.type, (dist.get_world_size(),))
        model = build_fsdp_llama(_cfg(), dev, torch.float32, mesh=mesh)
    else:
        model = Llama(_cfg()).to(dev)
    opt = _with_adamw(model)
    for src in ("sync", "async"):
        _zero_(model, opt)
        Snapshot(f"{tmp}/{src}").restore({"model": model, "optim": opt})
        _check(model, opt, ref, (target, src))
    # read_object of 2-D-sharded entries into plain tensors, with and without
    # a memory budget (tiled reads)
    for name in ("layers.0.attention.wq.weight", "layers.1.feed_forward.w2.weight",
                 "tok_embeddings.weight"):
        for budget in (None, 2048):
            plain = torch.zeros_like(ref[f"m/{name}"]).to(dev)
            Snapshot(f"{tmp}/async").read_object(f"0/model/{name}", obj_out=plain,
                                                 memory_budget_bytes=budget)
            assert torch.equal(plain.cpu(), ref[f"m/{name}"]), (name, budget)


@pytest.mark.multiproc
@pytest.mark.slow  # 25 s of CPU; its GPU twin runs in every GPU suite
def test_fsdp_over_tp_save_and_reshard(tmp_path):
    run_distributed(_save_worker, 4, str(tmp_path))
    for target in ("2d_same", "2d_swapped", "fsdp"):
        run_distributed(_restore_worker, 4, str(tmp_path), target)
    run_distributed(_restore_worker, 1, str(tmp_path), "plain")


@pytest.mark.gpu
def test_fsdp_over_tp_save_and_reshard_gpu(gpu, tmp_path):
    """The same on HIP tensors (4 gloo ranks sharing cuda:0): strided-shard
    boxes are staged and scattered by the device path."""
    run_distributed(_save_worker, 4, str(tmp_path), "cuda:0", timeout=600)
    for target in ("2d_swapped", "fsdp"):
        run_distributed(_restore_worker, 4, str(tmp_path), target, "cuda:0", timeout=600)
    run_distributed(_restore_worker, 1, str(tmp_path), "plain", "cuda:0", timeout=600)


def _hsdp_worker(tmp: str):
    """HSDP: (replicate=2, shard=2) mesh -- each box is saved once (small
    boxes whole, by one replica); restore into a 1-D (4,) FSDP mesh."""
    import torch.distributed as dist
    from torch.distributed.device_mesh import init_device_mesh
    from torch.distributed.tensor import Replicate, Shard, distribute_tensor

    from hipsnapshot import Snapshot, StateDict

    mesh = init_device_mesh("cpu", (2, 2), mesh_dim_names=("rep", "shard"))
    torch.manual_seed(0)
    full = torch.randn(37, 11)
    dt = distribute_tensor(full, mesh, [Replicate(), Shard(0)])
    col = distribute_tensor(full, mesh, [Shard(1), Shard(0)])  # 2-D block layout
    Snapshot.take(f"{tmp}/hsdp", {"s": StateDict(w=dt, c=col)})
    man = Snapshot(f"{tmp}/hsdp").get_manifest()
    def boxes(name):
        return sorted((tuple(s.offsets), tuple(s.sizes)) for k, e in man.items()
                      if k.endswith(f"/s/{name}") for s in e.shards)

    assert boxes("w") == [((0, 0), (19, 11)), ((19, 0), (18, 11))], boxes("w")
    assert len(boxes("c")) == 4
    m1 = init_device_mesh("cpu", (dist.get_world_size(),))
    for src_key in ("w", "c"):
        out = distribute_tensor(torch.zeros_like(full), m1, [Shard(1)])
        Snapshot(f"{tmp}/hsdp").restore({"s": StateDict(**{src_key: out})})
        assert torch.equal(out.full_tensor(), full), src_key


@pytest.mark.multiproc
def test_hsdp_and_block_layouts(tmp_path):
    run_distributed(_hsdp_worker, 4, str(tmp_path))


def _hsdp_balance_worker(tmp: str, shape):
    """HSDP on a ``shape`` = (replicas, shards) mesh: every rank writes about
    the same bytes (the replicas split each box by rows), and the snapshot
    restores bitwise into the same mesh and into a 1-D FSDP mesh."""
    import torch.distributed as dist
    from torch.distributed.device_mesh import init_device_mesh
    from torch.distributed.tensor import Replicate, Shard, distribute_tensor

    from hipsnapshot import Snapshot, StateDict
    from hipsnapshot.snapshot import TakeStats

    mesh = init_device_mesh("cpu", tuple(shape), mesh_dim_names=("rep", "shard"))
    gen = torch.Generator().manual_seed(7)
    full = {f"w{i}": torch.randn(2048 + 8 * i, 512, generator=gen) for i in range(6)}
    full.update({f"norm{i}": torch.randn(512, generator=gen) for i in range(4)})
    full["emb"] = torch.randn(4099, 256, generator=gen).to(torch.bfloat16)
    dts = {k: distribute_tensor(v, mesh, [Replicate(), Shard(0)]) for k, v in full.items()}
    Snapshot.take(f"{tmp}/hsdp", {"m": StateDict(**dts)})
    written = [None] * dist.get_world_size()
    dist.all_gather_object(written, TakeStats.last["bytes"])
    total = sum(v.numel() * v.element_size() for v in full.values())
    assert abs(sum(written) - total) <= 0.01 * total, (written, total)
    mean = sum(written) / len(written)
    assert max(written) / mean <= 1.10, written
    # every element saved exactly once
    man = Snapshot(f"{tmp}/hsdp").get_manifest()
    for k, v in full.items():
        cover = torch.zeros(v.shape, dtype=torch.int32)
        for mk, e in man.items():
            if mk.endswith(f"/m/{k}"):
                for s in e.shards:
                    cover[tuple(slice(o, o + z) for o, z in zip(s.offsets, s.sizes))] += 1
        assert bool((cover == 1).all()), k
    same = {k: distribute_tensor(torch.zeros_like(v), mesh, [Replicate(), Shard(0)])
            for k, v in full.items()}
    Snapshot(f"{tmp}/hsdp").restore({"m": StateDict(**same)})
    m1 = init_device_mesh("cpu", (dist.get_world_size(),))
    flat = {k: distribute_tensor(torch.zeros_like(v), m1, [Shard(0)]) for k, v in full.items()}
    Snapshot(f"{tmp}/hsdp").restore({"m": StateDict(**flat)})
    for k, v in full.items():
        assert torch.equal(same[k].full_tensor(), v), k
        assert torch.equal(flat[k].full_tensor(), v), k


@pytest.mark.multiproc
@pytest.mark.parametrize("shape", [(2, 2), (2, 4)], ids=["2x2", "2x4"])
def test_hsdp_write_load_is_balanced(tmp_path, shape):
    run_distributed(_hsdp_balance_worker, shape[0] * shape[1], str(tmp_path), list(shape),
                    timeout=300)
