"""Embedding-table resharding matrix (the reference's TorchRec GPU test).

Reference: `/root/reference/tests/gpu_tests/test_torchrec.py:181-304` -- ROW /
COLUMN / TABLE-wise DistributedModelParallel tables, every src -> dst pair,
sync and async, ``override_max_shard_size_bytes`` below the smallest shard
(forced sub-division), ``read_object`` of each table into a plain tensor,
and the fused optimizer's state restored across layouts.

Here the tables are ``hipsnapshot.models.dlrm`` DTensors (TorchRec is not
installable): row = ``Shard(0)``, column = ``Shard(1)``, table = whole table
on one rank's single-rank submesh.  The optimizer is Adagrad over the tables
(its ``sum`` state has each table's layout).  Values are compared BITWISE
against full tables generated from fixed seeds on every rank.

* CPU: 2 gloo ranks (``multiproc``);
* GPU: 2 gloo ranks sharing ``cuda:0`` (``gpu``): every restore goes through
  the device scatter path (pinned read -> H2D -> ``hs_copy_nd`` into the
  strided column / row regions).
"""

import itertools

import pytest
import torch

from hipsnapshot.utils.test_utils import run_distributed

TABLES = [96, 77, 50]
DIM = 24


def _full(kind: str, i: int, n: int) -> torch.Tensor:
    g = torch.Generator().manual_seed(1000 * i + {"w": 1, "sum": 2}[kind])
    return torch.rand(n, DIM, generator=g)


def _box_slices(b):
    return tuple(slice(o, o + s) for o, s in zip(b.offsets, b.sizes))


def _fill(model, opt, salt: int = 0) -> None:
    """Every local box of every table / optimizer state gets its slice of
    the seeded full table (+ salt)."""
    from hipsnapshot.io.sharded import local_boxes

    with torch.no_grad():
        for i, t in enumerate(model.tables):
            for b in local_boxes(t.weight):
                b.tensor.copy_(_full("w", i, t.num_embeddings)[_box_slices(b)] + salt)
            st = opt.state[t.weight]
            for b in local_boxes(st["sum"]):
                b.tensor.copy_(_full("sum", i, t.num_embeddings)[_box_slices(b)] + salt)


def _check(model, opt, tag) -> None:
    from hipsnapshot.io.sharded import local_boxes

    for i, t in enumerate(model.tables):
        for b in local_boxes(t.weight):
            want = _full("w", i, t.num_embeddings)[_box_slices(b)]
            assert torch.equal(b.tensor.cpu(), want), (tag, "w", i, b.offsets)
        for b in local_boxes(opt.state[t.weight]["sum"]):
            want = _full("sum", i, t.num_embeddings)[_box_slices(b)]
            assert torch.equal(b.tensor.cpu(), want), (tag, "sum", i, b.offsets)


def _smallest_shard_bytes(model) -> int:
    from hipsnapshot.io.sharded import local_boxes

    sizes = [b.tensor.numel() * b.tensor.element_size()
             for t in model.tables for b in local_boxes(t.weight)]
    return min(sizes) if sizes else 1 << 30


def _matrix_worker(tmp: str, device: str, batching: bool) -> None:
    import torch.distributed as dist
    from torch.distributed.device_mesh import init_device_mesh

    from hipsnapshot import Snapshot
    from hipsnapshot.knobs import override_is_batching_disabled, override_max_shard_size_bytes
    from hipsnapshot.models.dlrm import DLRM, SHARDINGS

    import faulthandler
    import sys
    import time

    # a hang prints every thread's stack instead of waiting for the runner
    faulthandler.dump_traceback_later(240, exit=True)
    dev = torch.device(device)
    if dev.type == "cuda":  # every rank shares this GPU (not LOCAL_RANK's)
        torch.cuda.set_device(dev)
    mesh = init_device_mesh(dev.type, (dist.get_world_size(),))
    ws = dist.get_world_size()
    cases = list(itertools.product(SHARDINGS, SHARDINGS, (False, True)))
    t0 = time.monotonic()
    with override_is_batching_disabled(not batching):
        for n, (src_kind, dst_kind, use_async) in enumerate(cases):
            src = DLRM(TABLES, dim=DIM, device=dev, mesh=mesh, sharding=src_kind)
            opt = src.make_optimizer()
            _fill(src, opt)
            # every rank agrees on the limit: half the smallest shard anywhere
            smallest = torch.tensor([_smallest_shard_bytes(src)], dtype=torch.int64)
            dist.all_reduce(smallest, op=dist.ReduceOp.MIN)
            path = f"{tmp}/c{n}"
            app = {"dlrm": src, "optim": opt}
            with override_max_shard_size_bytes(int(smallest.item()) // 2 - 1):
                if use_async:
                    snap = Snapshot.async_take(path, app).wait()
                else:
                    snap = Snapshot.take(path, app)
            man = snap.get_manifest()
            n_shards = sum(len(e.shards) for k, e in man.items()
                           if k.endswith("tables.0.weight") and hasattr(e, "shards"))
            assert n_shards >= 2 * (ws if src_kind != "table" else 1), (src_kind, n_shards)
            dst = DLRM(TABLES, dim=DIM, device=dev, mesh=mesh, sharding=dst_kind)
            dopt = dst.make_optimizer()
            _fill(dst, dopt, salt=5)  # different values everywhere
            snap.restore({"dlrm": dst, "optim": dopt})
            tag = (src_kind, dst_kind, use_async, batching)
            _check(dst, dopt, tag)
            if dist.get_rank() == 0:
                print(f"dlrm case {n} {tag} ok at {time.monotonic() - t0:.1f}s", file=sys.stderr,
                      flush=True)
            # read_object of every table (sharded entry) into a plain tensor
            for i, rows in enumerate(TABLES):
                for out_dev in {dev, torch.device("cpu")}:
                    plain = torch.zeros(rows, DIM, device=out_dev)
                    snap.read_object(f"0/dlrm/tables.{i}.weight", obj_out=plain)
                    assert torch.equal(plain.cpu(), _full("w", i, rows)), (tag, i, out_dev)
    faulthandler.cancel_dump_traceback_later()


@pytest.mark.multiproc
@pytest.mark.parametrize("batching", [True, False])
def test_dlrm_resharding_matrix_cpu(tmp_path, batching):
    run_distributed(_matrix_worker, 2, str(tmp_path), "cpu", batching, timeout=600)


@pytest.mark.gpu
@pytest.mark.parametrize("batching", [True, False])
def test_dlrm_resharding_matrix_gpu(gpu, tmp_path, batching):
    run_distributed(_matrix_worker, 2, str(tmp_path), "cuda:0", batching, backend="gloo",
                    timeout=300)


def _forward_worker(device: str) -> None:
    """The three layouts compute the same forward (same full tables)."""
    import torch.distributed as dist
    from torch.distributed.device_mesh import init_device_mesh

    from hipsnapshot.models.dlrm import DLRM, SHARDINGS

    dev = torch.device(device)
    mesh = init_device_mesh(dev.type, (dist.get_world_size(),))
    g = torch.Generator().manual_seed(3)
    dense = torch.rand(4, 13, generator=g).to(dev)
    sparse = [(torch.randint(0, n, (8,), generator=g).to(dev),
               torch.tensor([0, 2, 5, 6]).to(dev)) for n in TABLES]
    outs, ref = [], None
    for kind in SHARDINGS:
        m = DLRM(TABLES, dim=DIM, device=dev, mesh=mesh, sharding=kind)
        _fill(m, m.make_optimizer())
        if ref is None:
            ref = m
        else:  # same dense MLPs
            m.bottom.load_state_dict(ref.bottom.state_dict())
            m.top.load_state_dict(ref.top.state_dict())
        outs.append(m(dense, sparse))
    assert torch.allclose(outs[0], outs[1], atol=1e-5) and torch.allclose(outs[0], outs[2],
                                                                          atol=1e-5)


@pytest.mark.multiproc
def test_dlrm_layouts_same_forward_cpu():
    run_distributed(_forward_worker, 2, "cpu")
