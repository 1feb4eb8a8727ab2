"""Worker bodies for multi-process tests (module-level so spawn can import them)."""

import os
import time
from datetime import timedelta

import torch
import torch.distributed as dist

from hipsnapshot import Snapshot, StateDict
from hipsnapshot.parallel.comm import Comm
from hipsnapshot.utils.test_utils import assert_state_dict_eq


def _ddp_model(seed: int):
    torch.manual_seed(seed)
    return torch.nn.Sequential(torch.nn.Linear(16, 32), torch.nn.ReLU(), torch.nn.Linear(32, 4))


def ddp_take(path: str, chunk_bytes=None):
    from hipsnapshot.knobs import override_max_chunk_size_bytes

    rank = dist.get_rank()
    model = torch.nn.parallel.DistributedDataParallel(_ddp_model(0))
    per_rank = StateDict(rank=rank, t=torch.full((4,), float(rank)))
    app = {"model": model, "per_rank": per_rank}
    if chunk_bytes:
        with override_max_chunk_size_bytes(chunk_bytes):
            Snapshot.take(path, app)
    else:
        Snapshot.take(path, app)


def ddp_restore(path: str, saved_world: int):
    rank = dist.get_rank()
    model = torch.nn.parallel.DistributedDataParallel(_ddp_model(100 + rank))
    per_rank = StateDict(rank=-1)
    snap = Snapshot(path)
    snap.restore({"model": model, "per_rank": per_rank})
    ref = _ddp_model(0)
    assert_state_dict_eq(model.module.state_dict(), ref.state_dict())
    if rank < saved_world:
        assert per_rank["rank"] == rank and torch.equal(per_rank["t"], torch.full((4,), float(rank)))
    else:
        assert per_rank["rank"] == -1  # new rank: per-rank state is not available
    man = snap.get_manifest()
    # replicated entries are stored once, under rank 0
    assert any(k.startswith("0/model/") for k in man)
    assert not any(k.startswith("1/model/") for k in man)
    rep = [e for k, e in man.items() if k.startswith("0/model/") and hasattr(e, "location")]
    assert all(e.replicated for e in rep)


def write_load_balance(path: str):
    """Replicated big tensors must be spread over ranks by the partitioner."""
    from hipsnapshot.knobs import override_is_batching_disabled

    rank = dist.get_rank()
    sd = StateDict({f"w{i}": torch.full((1000 * (i + 1),), float(i)) for i in range(8)})
    with override_is_batching_disabled(True):
        Snapshot.take(path, {"sd": sd}, replicated=["**"])
    dist.barrier()
    if rank == 0:
        man = Snapshot(path).get_manifest()
        assert all(man[f"0/sd/w{i}"].replicated for i in range(8))
        assert all(man[f"0/sd/w{i}"].location.startswith("replicated/") for i in range(8))
    out = StateDict({f"w{i}": torch.zeros(1000 * (i + 1)) for i in range(8)})
    Snapshot(path).restore({"sd": out})
    for i in range(8):
        assert torch.equal(out[f"w{i}"], torch.full((1000 * (i + 1),), float(i)))


def partition_plan_check():
    from hipsnapshot.parallel.partitioner import partition_write_reqs
    from hipsnapshot.io.preparer import prepare_write
    from hipsnapshot.knobs import override_max_chunk_size_bytes

    comm = Comm()
    rank = comm.get_rank()
    ws = comm.get_world_size()
    entries, reqs = {}, {}
    with override_max_chunk_size_bytes(4000):
        for i in range(6):
            t = torch.ones(1000 * (i + 1))
            e, w = prepare_write(t, f"sd/t{i}", rank, replicated=True)
            entries[f"sd/t{i}"], reqs[f"sd/t{i}"] = e, w
    new_entries, new_reqs = partition_write_reqs(entries, reqs, comm)
    mine = sum(len(v) for v in new_reqs.values())
    gathered = [None] * ws
    comm.all_gather_object(gathered, (mine, sorted(new_reqs)))
    total = sum(len(v) for v in reqs.values())
    assert sum(g[0] for g in gathered) == total, gathered
    # balanced within one unit (chunks are ~4000 B each)
    counts = [g[0] for g in gathered]
    assert max(counts) - min(counts) <= 2, counts


def fsdp_take(path: str):
    from torch.distributed.device_mesh import init_device_mesh
    from hipsnapshot.models.llama import LlamaConfig, build_fsdp_llama

    mesh = init_device_mesh("cpu", (dist.get_world_size(),))
    model = build_fsdp_llama(LlamaConfig.tiny(), torch.device("cpu"), torch.float32, mesh=mesh)
    Snapshot.take(path, {"model": model})
    full = {k: v.full_tensor() for k, v in model.state_dict().items()}
    if dist.get_rank() == 0:
        torch.save(full, path + "_ref.pt")


def fsdp_take_reusing_plan(path: str):
    """Several takes of FSDP2 (DTensor) state with the plan cache active on
    every rank (host tensors marked resident): later takes reuse the plan,
    each snapshot restores to the values it was taken with."""
    from torch.distributed.device_mesh import init_device_mesh

    from hipsnapshot.engine import plan_cache
    from hipsnapshot.models.llama import LlamaConfig, build_fsdp_llama

    plan_cache.is_resident = lambda obj: hasattr(obj, "_local_tensor")
    plan_cache.clear()
    mesh = init_device_mesh("cpu", (dist.get_world_size(),))
    model = build_fsdp_llama(LlamaConfig.tiny(), torch.device("cpu"), torch.float32, mesh=mesh)
    refs = []
    for i in range(3):
        with torch.no_grad():
            for p in model.parameters():
                p._local_tensor.add_(1.0)
        Snapshot.take(f"{path}_{i}", {"model": model, "progress": StateDict(step=i)})
        refs.append({k: v.full_tensor().clone() for k, v in model.state_dict().items()})
    assert plan_cache.stats["hits"] == 2, plan_cache.stats
    for i in range(3):
        for p in model.parameters():
            p._local_tensor.zero_()
        prog = StateDict(step=-1)
        Snapshot(f"{path}_{i}").restore({"model": model, "progress": prog})
        assert prog["step"] == i
        for k, v in model.state_dict().items():
            assert torch.equal(v.full_tensor(), refs[i][k]), (i, k)


def fsdp_restore(path: str):
    from torch.distributed.device_mesh import init_device_mesh
    from hipsnapshot.models.llama import Llama, LlamaConfig
    from torch.distributed.fsdp import fully_shard

    ws = dist.get_world_size()
    mesh = init_device_mesh("cpu", (ws,))
    with torch.device("meta"):
        model = Llama(LlamaConfig.tiny())
    for layer in model.layers:
        fully_shard(layer, mesh=mesh)
    fully_shard(model, mesh=mesh)
    model.to_empty(device="cpu")
    for p in model.parameters():
        p._local_tensor.zero_()
    # FSDP2's load hooks are known no-ops after an in-place restore: the
    # module's load_state_dict (a self-copy of every DTensor) is skipped
    import torch.nn as nn

    from hipsnapshot.snapshot import _plain_module_load

    assert _plain_module_load(model)
    calls = []
    orig = nn.Module.load_state_dict
    nn.Module.load_state_dict = lambda self, *a, **k: calls.append(1) or orig(self, *a, **k)
    try:
        # verified: the shard blobs of every saving rank (their checksum
        # files), whole or as byte ranges of another world size's shards
        Snapshot(path).restore({"model": model}, verify=True)
    finally:
        nn.Module.load_state_dict = orig
    assert not calls
    ref = torch.load(path + "_ref.pt", weights_only=True)
    for k, v in model.state_dict().items():
        assert torch.equal(v.full_tensor(), ref[k]), k
    # read_object of a sharded entry into a plain tensor (whole global tensor)
    w = torch.zeros_like(ref["layers.0.attention.wq.weight"])
    Snapshot(path).read_object("0/model/layers.0.attention.wq.weight", obj_out=w, verify=True)
    assert torch.equal(w, ref["layers.0.attention.wq.weight"])


def _fsdp_adamw(seed: int):
    from torch.distributed.device_mesh import init_device_mesh
    from hipsnapshot.models.llama import LlamaConfig, build_fsdp_llama

    mesh = init_device_mesh("cpu", (dist.get_world_size(),))
    torch.manual_seed(seed)
    model = build_fsdp_llama(LlamaConfig.tiny(), torch.device("cpu"), torch.float32, mesh=mesh)
    return model, torch.optim.AdamW(model.parameters(), lr=1e-3, weight_decay=0.1)


def _full_optim_state(optim):
    out = {}
    for i, st in optim.state_dict()["state"].items():
        for name, v in st.items():
            out[(i, name)] = v.full_tensor() if hasattr(v, "full_tensor") else v.clone()
    return out


def fsdp_optim_take(path: str):
    """FSDP2 + AdamW after two steps: model and (sharded) optimizer state."""
    model, optim = _fsdp_adamw(0)
    for _ in range(2):
        tokens = torch.randint(0, 256, (2, 16))
        model(tokens).float().logsumexp(-1).mean().backward()
        optim.step()
        optim.zero_grad()
    Snapshot.take(path, {"model": model, "optim": optim})
    ref = {"model": {k: v.full_tensor() for k, v in model.state_dict().items()},
           "optim": _full_optim_state(optim)}
    if dist.get_rank() == 0:
        torch.save(ref, path + "_ref.pt")


def fsdp_optim_restore_fresh(path: str):
    """A fresh process (any world size) restores into a model and an AdamW
    that never stepped: the sharded optimizer state has no tensors to land in
    until hipsnapshot materializes them; the parameters must come out as
    saved, not moved by that zero step."""
    model, optim = _fsdp_adamw(1)
    assert not optim.state
    Snapshot(path).restore({"model": model, "optim": optim})
    ref = torch.load(path + "_ref.pt", weights_only=True)
    for k, v in model.state_dict().items():
        assert torch.equal(v.full_tensor(), ref["model"][k]), k
    got = _full_optim_state(optim)
    assert set(got) == set(ref["optim"])
    for k, v in got.items():
        assert torch.equal(v, ref["optim"][k]), k
    assert all(p.grad is None for p in model.parameters())
    assert optim.param_groups[0]["lr"] == 1e-3


class FaultyPlugin:
    pass


def async_take_ok(path: str):
    rank = dist.get_rank()
    t = torch.full((1000,), float(rank))
    sd = StateDict(t=t, step=rank)
    pending = Snapshot.async_take(path, {"sd": sd})
    t.fill_(-1)  # must not leak into the snapshot
    snap = pending.wait()
    assert pending.done()
    out = StateDict()
    snap.restore({"sd": out})
    assert torch.equal(out["t"], torch.full((1000,), float(rank))) and out["step"] == rank


def async_take_faulty(path: str):
    import asyncio
    from unittest import mock

    from hipsnapshot.storage.fs import FSStoragePlugin

    rank = dist.get_rank()

    class Faulty(FSStoragePlugin):
        async def write(self, write_io):
            if rank == 1 and not write_io.path.startswith(".snapshot"):
                await asyncio.sleep(0.2)
                raise OSError("injected failure")
            await super().write(write_io)

    with mock.patch("hipsnapshot.storage.fs.FSStoragePlugin", Faulty):
        pending = Snapshot.async_take(path, {"sd": StateDict(t=torch.ones(100) * rank)})
        try:
            pending.wait()
            raised = False
        except RuntimeError as e:
            raised = True
            assert "injected failure" in str(e) or "encountered error" in str(e), str(e)
    assert raised, "every rank must observe the failure"
    dist.barrier()
    assert not os.path.exists(os.path.join(path, ".snapshot_metadata"))


def async_take_staging_fault(path: str):
    """Rank 1 fails while staging, after the metadata gather: rank 0's commit
    thread must fail promptly through the barrier, not after its timeout."""
    import time
    from datetime import timedelta
    from unittest import mock

    from hipsnapshot.snapshot import PendingSnapshot

    rank = dist.get_rank()

    def boom(*a, **k):
        raise OSError("injected staging failure")

    PendingSnapshot.DEFAULT_BARRIER_TIMEOUT = timedelta(seconds=120)
    sd = {"sd": StateDict(t=torch.ones(100) * rank)}
    t0 = time.monotonic()
    if rank == 1:
        with mock.patch("hipsnapshot.snapshot.sync_execute_write_reqs", boom):
            try:
                Snapshot.async_take(path, sd)
                raise AssertionError("async_take should have raised")
            except OSError as e:
                assert "injected staging failure" in str(e)
    else:
        pending = Snapshot.async_take(path, sd)
        try:
            pending.wait()
            raise AssertionError("rank 0 must observe rank 1's failure")
        except RuntimeError as e:
            assert "injected staging failure" in str(e), str(e)
        assert time.monotonic() - t0 < 60, "failure was not propagated through the barrier"
    dist.barrier()
    assert not os.path.exists(os.path.join(path, ".snapshot_metadata"))


def linear_barrier(prefix: str, skip_arrive_rank: int = -1, error_rank: int = -1):
    from hipsnapshot.parallel.store import LinearBarrier, get_or_create_store

    comm = Comm()
    store = get_or_create_store(comm)
    rank, ws = comm.get_rank(), comm.get_world_size()
    b = LinearBarrier(prefix, store, rank, ws, leader_rank=0)
    if rank == error_rank:
        b.report_error("boom")
        return
    if rank == skip_arrive_rank:
        return
    clean_run = error_rank < 0 and skip_arrive_rank < 0
    if clean_run:
        n0 = store.num_keys()
        dist.barrier()
    # a skipped arrival only has to time out: 1 s; clean runs keep slack
    to = timedelta(seconds=1 if skip_arrive_rank >= 0 else 3)
    try:
        b.arrive(timeout=to)
        b.depart(timeout=to)
        assert error_rank < 0 and skip_arrive_rank < 0
        dist.barrier()
        # the barrier cleaned up after itself (num_keys also counts the
        # c10d barrier's own bookkeeping keys: compare after a barrier each)
        assert store.num_keys() <= n0 + 2, (store.num_keys(), n0)
        for r in range(ws):
            assert not store.check([f"{prefix}_{r}"]), r
        assert not store.check([f"{prefix}_departed"])
    except RuntimeError as e:
        assert error_rank >= 0 or skip_arrive_rank >= 0, e
        if error_rank >= 0:
            assert "boom" in str(e)
    except Exception as e:  # store timeout
        assert skip_arrive_rank >= 0, e


def comm_collectives():
    comm = Comm()
    rank, ws = comm.get_rank(), comm.get_world_size()
    big = "x" * (200_000 * (rank + 1))  # > 64 KiB frame -> second round
    out = [None] * ws
    comm.all_gather_object(out, {"r": rank, "big": big})
    for r in range(ws):
        assert out[r]["r"] == r and len(out[r]["big"]) == 200_000 * (r + 1)
    small = [None] * ws
    comm.all_gather_object(small, rank * 10)
    assert small == [r * 10 for r in range(ws)]
    obj = [f"from0-{rank}"]
    comm.broadcast_object_list(obj, src=0)
    assert obj == ["from0-0"]
    res = [None]
    comm.scatter_object_list(res, [f"s{r}" for r in range(ws)] if rank == 0 else None, src=0)
    assert res[0] == f"s{rank}"


def replication_globs(path: str):
    """replicated = glob matched on ALL ranks, present on all ranks, not sharded."""
    rank = dist.get_rank()
    sd = StateDict(common=torch.ones(4), only_rank0=torch.ones(2),
                   per=torch.full((3,), float(rank)), nested={"a": torch.zeros(2), "b": 1})
    if rank != 0:
        del sd["only_rank0"]
    # rank 1 passes an extra glob that rank 0 does not: it must be ignored
    globs = ["sd/common", "sd/only_rank0", "sd/nested/*"] + (["sd/per"] if rank == 1 else [])
    Snapshot.take(path, {"sd": sd}, replicated=globs)
    man = Snapshot(path).get_manifest()
    assert man["0/sd/common"].replicated and man["0/sd/nested/a"].replicated
    assert man["0/sd/nested/b"].replicated  # primitives can be replicated too
    assert not man["0/sd/only_rank0"].replicated  # absent on rank 1
    assert not man["0/sd/per"].replicated and "1/sd/per" in man
    assert "1/sd/common" not in man  # replicated entries live under rank 0 only


def ddp_infer_replication(path: str, ignore: bool):
    rank = dist.get_rank()
    torch.manual_seed(0)
    inner = torch.nn.Sequential(torch.nn.Linear(4, 4), torch.nn.Linear(4, 2))
    if ignore:
        torch.nn.parallel.DistributedDataParallel._set_params_and_buffers_to_ignore_for_model(
            inner, ["1.weight"])
    model = torch.nn.parallel.DistributedDataParallel(inner)
    Snapshot.take(path, {"ddp": model})
    man = Snapshot(path).get_manifest()
    if ignore:
        assert not man["0/ddp/module.1.weight"].replicated
        assert f"{1}/ddp/module.1.weight" in man
        assert man["0/ddp/module.0.weight"].replicated
    else:
        assert all(e.replicated for k, e in man.items() if hasattr(e, "location"))


def committed_on_return(path):
    """take() returns on every rank only once .snapshot_metadata exists."""
    import os

    import torch

    from hipsnapshot import Snapshot, StateDict

    rank = torch.distributed.get_rank()
    for i in range(5):
        p = f"{path}_{i}"
        sd = StateDict(t=torch.full((1000,), float(rank + i)), step=i)
        Snapshot.take(p, {"sd": sd})
        assert os.path.exists(os.path.join(p, ".snapshot_metadata")), (rank, i)
        out = StateDict(t=torch.zeros(1000), step=-1)
        Snapshot(p).restore({"sd": out})
        assert out["step"] == i and torch.equal(out["t"], torch.full((1000,), float(rank + i)))


def distributed_verify(path: str):
    """Every rank checks its share of the blobs; all get the merged report,
    and a corrupted blob shows up in it whichever rank checked it."""
    rank = dist.get_rank()
    ws = dist.get_world_size()
    torch.manual_seed(rank)
    sd = StateDict(w=torch.randn(1000 + rank, 17), **{f"t{i}": torch.randn(300, 40)
                                                    for i in range(6)})
    snap = Snapshot.take(path, {"sd": sd}, replicated=[])
    rep = snap.verify(distributed=True)
    assert rep.ok and rep.checked == rep.blobs > 0, rep
    whole = snap.verify()  # local, single-process
    assert whole.blobs == rep.blobs and whole.ok
    dist.barrier()
    if rank == 0:
        victim = sorted(
            os.path.join(d, f) for d, _, fs in os.walk(path) for f in fs
            if not os.path.relpath(os.path.join(d, f), path).startswith(".snapshot"))[-1]
        with open(victim, "r+b") as f:
            f.seek(3)
            b = f.read(1)
            f.seek(3)
            f.write(bytes([b[0] ^ 0xFF]))
    dist.barrier()
    rep = snap.verify(distributed=True)
    assert not rep.ok and len(rep.mismatched) == 1, rep
    assert ws > 1


def async_metadata_via_store(path: str):
    """async_take exchanges manifests through the c10d store in the commit
    thread (no collective before it returns): replicated (DDP), sharded
    (DTensor) and per-rank entries all land in the metadata, identical in
    shape to a sync take's, and the store keys are cleaned up."""
    from torch.distributed.device_mesh import init_device_mesh
    from torch.distributed.tensor import Shard, distribute_tensor

    from unittest import mock

    import hipsnapshot.snapshot as snapmod
    from hipsnapshot.parallel.store import get_or_create_store

    rank, ws = dist.get_rank(), dist.get_world_size()
    mesh = init_device_mesh("cpu", (ws,))
    torch.manual_seed(0)
    full = torch.randn(33, 7)
    ddp = torch.nn.parallel.DistributedDataParallel(_ddp_model(0))
    app = {"ddp": ddp, "sd": StateDict(own=torch.full((5,), float(rank)),
                                       dt=distribute_tensor(full, mesh, [Shard(0)]),
                                       step=rank)}
    Snapshot.take(path + "_sync", app)
    used = []
    orig_key = snapmod._manifest_key

    def spy(*a):
        used.append(orig_key(*a))
        return used[-1]

    with mock.patch.object(snapmod, "_manifest_key", spy):
        pending = Snapshot.async_take(path + "_async", app)
        snap = pending.wait()
    m_sync = Snapshot(path + "_sync").get_manifest()
    m_async = snap.get_manifest()
    assert sorted(m_sync) == sorted(m_async), set(m_sync) ^ set(m_async)
    for k in m_sync:
        assert type(m_sync[k]) is type(m_async[k]), k
    store = get_or_create_store(Comm())
    dist.barrier()
    # every rank published its manifest; rank 0 removed them after assembling
    assert used
    for k in used:
        assert not store.check([k]), k
    out = {"ddp": torch.nn.parallel.DistributedDataParallel(_ddp_model(1)), "sd": StateDict(own=torch.zeros(5),
                                                 dt=distribute_tensor(torch.zeros_like(full),
                                                                      mesh, [Shard(0)]),
                                                 step=-1)}
    snap.restore(out)
    assert out["sd"]["step"] == rank
    assert torch.equal(out["sd"]["own"], torch.full((5,), float(rank)))
    assert torch.equal(out["sd"]["dt"].full_tensor(), full)
    for a, b in zip(out["ddp"].parameters(), ddp.parameters()):
        assert torch.equal(a, b)


class _CollectiveStateful:
    """A stateful whose state_dict() runs a collective (unknown kind)."""

    def __init__(self):
        self.t = torch.ones(3)

    def state_dict(self):
        x = torch.ones(1)
        dist.all_reduce(x)
        return {"t": self.t, "n": int(x.item())}

    def load_state_dict(self, sd):
        self.t.copy_(sd["t"])


def state_dict_barriers():
    """Per-key barriers run only when some rank's state_dict() may issue a
    collective: StateDict/module-only app states skip them."""
    import tempfile
    from unittest import mock

    from hipsnapshot.parallel.comm import Comm as C

    calls = []
    orig = C.barrier

    def counting(self, *a, **k):
        calls.append(1)
        return orig(self, *a, **k)

    d = tempfile.mkdtemp() if dist.get_rank() == 0 else None
    box = [d]
    dist.broadcast_object_list(box)
    with mock.patch.object(C, "barrier", counting):
        app = {"a": StateDict(x=torch.ones(2)), "b": torch.nn.Linear(2, 2),
               "c": StateDict(y=1)}
        Snapshot.take(box[0] + "/p", app)
        n_local = len(calls)
        calls.clear()
        app["d"] = _CollectiveStateful()
        Snapshot.take(box[0] + "/q", app)
        n_coll = len(calls)
    # commit barriers only vs + one per app-state key (4 keys)
    assert n_coll - n_local == 4, (n_local, n_coll)


def rebalance_take(path: str):
    """Rank 0 owns most of the bytes; with rebalancing, its blobs are written
    by the idle ranks (their checksum files list them), the manifest is
    unchanged and every rank restores bitwise."""
    import json

    from hipsnapshot.knobs import override_knob, override_slab_size_threshold_bytes
    from hipsnapshot.verify import verify_snapshot

    rank, ws = dist.get_rank(), dist.get_world_size()
    torch.manual_seed(rank)
    n = 8 if rank == 0 else 1
    sd = StateDict(**{f"t{i}": torch.randn(64 * 1024 + 7 * i) for i in range(n)}, r=rank)
    with override_knob("REBALANCE", "1"), override_knob("REBALANCE_HOST", "1"), \
            override_slab_size_threshold_bytes(1024):
        Snapshot.take(path, {"sd": sd})
    dist.barrier()
    if rank == 0:
        assert verify_snapshot(path).ok
        written = {}
        for r in range(ws):
            doc = json.load(open(os.path.join(path, ".snapshot_checksums", str(r))))
            written[r] = set(doc["blobs"])
        moved = [p for r in range(1, ws) for p in written[r] if p.startswith("0/")]
        assert moved, written  # idle ranks wrote some of rank 0's blobs
    out = StateDict(**{f"t{i}": torch.zeros(64 * 1024 + 7 * i) for i in range(n)}, r=-1)
    Snapshot(path).restore({"sd": out})
    assert out["r"] == rank
    for i in range(n):
        assert torch.equal(out[f"t{i}"], sd[f"t{i}"]), i


def _register_guarded_fs(delay_s: float) -> None:
    """``guardfs://``: the FS plugin, except that writing a blob while the
    path still holds a ``.snapshot_metadata`` raises (a crash there would
    leave a committed snapshot with torn blobs) and rank 0's delete of the
    old metadata is delayed, so a rank that wrote before the uncommit would
    be caught."""
    from hipsnapshot.storage import fs as fsmod
    from hipsnapshot.storage.registry import register_storage_plugin

    class GuardedFS(fsmod.FSStoragePlugin):
        def _committed(self) -> bool:
            return os.path.exists(os.path.join(self.root, ".snapshot_metadata"))

        async def write(self, write_io):
            if write_io.path != ".snapshot_metadata" and self._committed():
                raise AssertionError(f"rank {dist.get_rank()} wrote {write_io.path} "
                                     "while the previous commit still existed")
            return await super().write(write_io)

        async def delete(self, path):
            if path == ".snapshot_metadata":
                time.sleep(delay_s)
            return await super().delete(path)

    register_storage_plugin("guardfs", lambda p, o: GuardedFS(root=p, storage_options=o))


def rewrite_never_overlaps_commit(path: str, delay_s: float = 1.0):
    """take / async_take into a path that holds a committed snapshot: every
    rank's blob writes start only after rank 0 removed the old commit."""
    from hipsnapshot.knobs import override_is_batching_disabled

    _register_guarded_fs(delay_s)
    rank = dist.get_rank()
    sd = StateDict({f"w{i}": torch.full((256 + 64 * i,), float(rank + i)) for i in range(4)})
    app = {"sd": sd}
    with override_is_batching_disabled(True):  # one write per tensor
        Snapshot.take(path, app)
        dist.barrier()
        for i in range(2):
            sd[f"w{i}"] += 1.0
            Snapshot.take("guardfs://" + path, app)
            pending = Snapshot.async_take("guardfs://" + path, app)
            pending.wait()
    out = StateDict({f"w{i}": torch.zeros(256 + 64 * i) for i in range(4)})
    Snapshot(path).restore({"sd": out})
    for k in out:
        assert torch.equal(out[k], sd[k]), k


def forced_collectives(path: str, out_json: str, use_cuda: bool):
    """``HIPSNAPSHOT_FORCE_COLLECTIVES=1`` in a one-rank group: every Comm
    collective (framed all-gather incl. its overflow round, broadcast,
    barrier, scatter), the store bootstrap broadcast, a self point-to-point
    exchange (RCCL), and a whole take / async_take / restore (the sync
    take's metadata gather runs on its helper thread beside staging) really
    issue their collectives.  Writes what it observed to ``out_json`` so the
    RCCL and gloo runs can be compared."""
    import json

    from hipsnapshot.parallel.comm import Comm
    from hipsnapshot.parallel.rebalance import p2p_exchange
    from hipsnapshot.parallel.store import create_store

    os.environ["HIPSNAPSHOT_FORCE_COLLECTIVES"] = "1"
    comm = Comm()
    assert comm.force and not comm.solo() and comm.get_world_size() == 1
    rank = comm.get_rank()
    nccl = "nccl" in str(comm.backend())
    res = {"backend": "nccl" if nccl else "gloo"}
    small = [None]
    comm.all_gather_object(small, {"rank": rank, "s": "x" * 100})
    res["small"] = small
    big_payload = bytes(range(256)) * 1024  # 256 KiB: the 64 KiB frame overflows
    big = [None]
    comm.all_gather_object(big, big_payload)
    assert big[0] == big_payload
    res["big_len"] = len(big[0])
    objs = ["some/path", {"x": 3}] if rank == 0 else [None, None]
    comm.broadcast_object_list(objs, src=0)
    res["bcast"] = objs
    comm.barrier()
    out = [None]
    comm.scatter_object_list(out, [["mine", rank]], src=0)
    res["scatter"] = out
    store = create_store(comm)  # rank 0 broadcasts the address: a collective
    store.set("forced_k", "v")
    res["store"] = store.get("forced_k").decode()
    if nccl:
        dev = torch.device("cuda", torch.cuda.current_device())
        src = torch.arange(1 << 20, dtype=torch.int32, device=dev)
        dst = torch.empty_like(src)
        p2p_exchange([(src, 0)], [(dst, 0)], comm)  # a rank is its own peer
        torch.cuda.synchronize()
        assert torch.equal(src, dst)
    if use_cuda:
        from torch.distributed.device_mesh import init_device_mesh

        from hipsnapshot.models.llama import LlamaConfig, build_fsdp_llama

        mesh = init_device_mesh("cuda", (1,))
        torch.manual_seed(0)
        m = build_fsdp_llama(LlamaConfig.tiny(), torch.device("cuda", torch.cuda.current_device()),
                             torch.bfloat16, mesh=mesh)

        def full(mod):
            return {k: v.full_tensor().clone() for k, v in mod.state_dict().items()}

        def zero(mod):
            for p in mod.parameters():
                p._local_tensor.zero_()
    else:
        torch.manual_seed(0)
        m = torch.nn.Sequential(torch.nn.Linear(64, 128), torch.nn.Linear(128, 8))

        def full(mod):
            return {k: v.clone() for k, v in mod.state_dict().items()}

        def zero(mod):
            with torch.no_grad():
                for p in mod.parameters():
                    p.zero_()
    ref = full(m)
    extra = StateDict(step=7)
    app = {"model": m, "extra": extra}
    s1 = Snapshot.take(path, app, replicated=["extra/**"])
    pending = Snapshot.async_take(path + "_a", app)
    s2 = pending.wait()
    keys = {}
    for tag, snap in (("take", s1), ("async", s2)):
        zero(m)
        extra["step"] = -1
        Snapshot(snap.path).restore(app)
        if use_cuda:
            torch.cuda.synchronize()
        got = full(m)
        for k, v in ref.items():
            assert torch.equal(got[k], v), (tag, k)
        assert extra["step"] == 7
        keys[tag] = sorted(Snapshot(snap.path).get_manifest().keys())
    res["manifest_keys"] = keys
    res["sha"] = {k: float(v.float().sum().item()) for k, v in sorted(ref.items())}
    with open(out_json, "w") as f:
        json.dump(res, f, sort_keys=True)
