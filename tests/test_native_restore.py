"""Native restore (engine/native_restore.py, csrc/hsrestore.cpp): every read
whose bytes land in HBM goes through one native job; the results must equal
the Python pipeline's bit for bit, for raw and HSZ1 blobs, batched slabs,
strided / narrowed / cast destinations and resharded DTensors; corrupt or
short files must raise."""

import os

import pytest
import torch

from hipsnapshot import Snapshot, StateDict
from hipsnapshot.knobs import override_knob

pytestmark = pytest.mark.gpu


def _state(gpu, seed=0):
    g = torch.Generator(device=gpu).manual_seed(seed)
    a = torch.randn(512, 256, device=gpu, generator=g)
    return StateDict(
        w=(torch.randn(1000, 300, device=gpu, generator=g) * 0.02).to(torch.bfloat16),
        big=(torch.randn(3000, 1024, device=gpu, generator=g) * 0.02).to(torch.bfloat16),
        t=a.t(),                                   # strided view, fp32
        col=a[:, 10:100],
        small=[torch.randn(i + 1000, device=gpu, generator=g) for i in range(20)],
        h=torch.randn(70_001, device=gpu, dtype=torch.float16, generator=g),
        i64=torch.arange(100_000, device=gpu),
        odd=torch.randn(3, 5, 7, device=gpu, generator=g)[:, 1:4, ::2],
    )


def _zeros_like_state(sd):
    out = {}
    for k, v in sd.items():
        if isinstance(v, list):
            out[k] = [torch.zeros_like(x) for x in v]
        else:
            out[k] = torch.zeros_like(v)
    return StateDict(**out)


def _eq(a, b):
    for k in a:
        if isinstance(a[k], list):
            assert all(torch.equal(x, y) for x, y in zip(a[k], b[k])), k
        else:
            assert torch.equal(a[k], b[k]), k


@pytest.mark.parametrize("compression", ["none", "hsz1"])
def test_native_restore_matches_python_pipeline(gpu, tmp_path, compression):
    from hipsnapshot.engine import native_restore

    src = _state(gpu)
    path = str(tmp_path / "s")
    Snapshot.take(path, {"sd": src}, compression=compression)
    outs = {}
    for flag in ("1", "0"):
        native_restore.last_stats.clear()
        dst = _zeros_like_state(src)
        with override_knob("NATIVE_RESTORE", flag):
            Snapshot(path).restore({"sd": dst})
        torch.cuda.synchronize()
        if flag == "1":
            # the native job ran and restored every tensor
            assert native_restore.last_stats.get("items", 0) > 0
        else:
            assert not native_restore.last_stats
        outs[flag] = dst
    _eq(outs["1"], src)
    _eq(outs["0"], src)


def test_native_restore_dtensor_resharding(gpu, tmp_path):
    """Row-sharded pieces restored into a different split (narrowed regions
    of several saved shards per destination) via the native job."""
    from hipsnapshot.utils.test_utils import run_distributed

    run_distributed(_reshard_worker, 2, str(tmp_path), timeout=600)


def _reshard_worker(root):
    import torch.distributed as dist
    from torch.distributed.device_mesh import init_device_mesh
    from torch.distributed.tensor import DTensor, Shard

    from hipsnapshot.engine import native_restore

    rank = dist.get_rank()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    mesh = init_device_mesh("cuda", (2,))  # all ranks share this GPU

    def dt(local, dim):  # no collectives (a "cuda" mesh group would be RCCL)
        return DTensor.from_local(local, mesh, [Shard(dim)], run_check=False)

    full = torch.arange(96 * 40, dtype=torch.float32, device=dev).reshape(96, 40)
    want = full[:, rank * 20:(rank + 1) * 20]
    for comp in ("none", "hsz1"):
        path = os.path.join(root, comp)
        Snapshot.take(path, {"sd": StateDict(x=dt(full[rank * 48:(rank + 1) * 48].clone(), 0))},
                      compression=comp)
        # restore column-sharded: every destination needs a narrow of both pieces
        for dtype in (torch.float32, torch.bfloat16):  # bf16: cast on the device (RNE)
            loc = torch.zeros(96, 20, device=dev, dtype=dtype)
            native_restore.last_stats.clear()
            Snapshot(path).restore({"sd": StateDict(x=dt(loc, 1))})
            torch.cuda.synchronize()
            assert native_restore.last_stats.get("items", 0) > 0
            assert torch.equal(loc, want.to(dtype)), (comp, dtype)


def test_native_restore_rejects_corrupt_frame_table(gpu, tmp_path):
    from hipsnapshot.knobs import override_is_batching_disabled
    from hipsnapshot.ops import codec, native

    big = (torch.randn(3000, 1024, device=gpu) * 0.02).to(torch.bfloat16)
    path = str(tmp_path / "c")
    with override_is_batching_disabled(True):
        Snapshot.take(path, {"sd": StateDict(big=big)}, compression="hsz1")
    f = os.path.join(path, "0", "sd", "big")
    blob = open(f, "rb").read()
    h = codec.parse_header(blob)
    with open(f, "r+b") as fh:  # frame 1 claims to end before it starts
        fh.seek(64 + 8 * 2)
        fh.write(int(h.offsets[1] - 64).to_bytes(8, "little"))
    out = StateDict(big=torch.zeros_like(big))
    with override_is_batching_disabled(True), pytest.raises(native.CorruptBlobError):
        Snapshot(path).restore({"sd": out})
    torch.cuda.synchronize()


def test_native_restore_short_file_raises(gpu, tmp_path):
    from hipsnapshot.knobs import override_is_batching_disabled

    big = torch.randn(1 << 20, device=gpu)
    path = str(tmp_path / "r")
    with override_is_batching_disabled(True):
        Snapshot.take(path, {"sd": StateDict(big=big)})
    f = os.path.join(path, "0", "sd", "big")
    with open(f, "r+b") as fh:
        fh.truncate(os.path.getsize(f) // 2)
    out = StateDict(big=torch.zeros_like(big))
    with override_is_batching_disabled(True), pytest.raises(OSError):
        Snapshot(path).restore({"sd": out})
    torch.cuda.synchronize()


def test_native_restore_device_budget_smaller_than_items(gpu, tmp_path):
    """Items larger than the device budget still go one at a time."""
    from hipsnapshot.engine import native_restore

    g = torch.Generator(device=gpu).manual_seed(9)
    # 8 MiB blobs under an 8 MiB budget (one or two in flight), and one
    # 32 MiB blob that exceeds it on its own (admitted when nothing else is)
    src = StateDict(**{f"t{i}": (torch.randn(1 << (22 if i != 3 else 24), device=gpu,
                                             generator=g) * 0.02).to(torch.bfloat16)
                       for i in range(6)})
    path = str(tmp_path / "b")
    Snapshot.take(path, {"sd": src}, compression="hsz1")
    dst = _zeros_like_state(src)
    with override_knob("RESTORE_DEVICE_BUDGET", str(8 << 20)), \
            override_knob("RESTORE_SLOT_BYTES", str(1 << 20)), \
            override_knob("RESTORE_SLOTS", "3"), override_knob("RESTORE_READERS", "5"):
        Snapshot(path).restore({"sd": dst})
    torch.cuda.synchronize()
    assert native_restore.last_stats.get("items", 0) == 6
    _eq(dst, src)


def test_native_restore_ring_wraps_when_empty(gpu, tmp_path):
    """A blob that fits the device ring only from its start, after an earlier
    blob left the (empty) ring's head past the middle: 5 MiB then 6 MiB
    under an 8 MiB ring (the second used to wait forever)."""
    from hipsnapshot.engine import native_restore
    from hipsnapshot.knobs import override_is_batching_disabled

    g = torch.Generator(device=gpu).manual_seed(5)
    src = StateDict(a=torch.randn(5 << 18, device=gpu, generator=g),
                    b=torch.randn(6 << 18, device=gpu, generator=g))
    path = str(tmp_path / "w")
    with override_is_batching_disabled(True):
        Snapshot.take(path, {"sd": src})
    for _ in range(2):  # ring reuse across jobs too
        dst = _zeros_like_state(src)
        with override_is_batching_disabled(True), \
                override_knob("RESTORE_DEVICE_BUDGET", str(8 << 20)), \
                override_knob("RESTORE_SLOT_BYTES", str(1 << 20)), \
                override_knob("RESTORE_SLOTS", "2"):
            Snapshot(path).restore({"sd": dst})
        torch.cuda.synchronize()
        assert native_restore.last_stats.get("items", 0) == 2
        _eq(dst, src)


def test_restore_plan_cache_hits_and_invalidates(gpu, tmp_path):
    """A second restore of the same snapshot into the same tensors reuses the
    native plan; a new take at the path, or a replaced tensor, plans again."""
    from hipsnapshot.engine import restore_cache

    restore_cache.clear()
    g = torch.Generator(device=gpu).manual_seed(2)
    sd = StateDict(a=(torch.randn(1 << 20, device=gpu, generator=g) * 0.02).to(torch.bfloat16),
                   b=torch.randn(300, 7, device=gpu, generator=g))
    path = str(tmp_path / "p")
    Snapshot.take(path, {"sd": sd}, compression="hsz1")
    want = {k: v.clone() for k, v in sd.items()}
    h0 = dict(restore_cache.stats)
    for _ in range(3):
        for v in sd.values():
            v.zero_()
        Snapshot(path).restore({"sd": sd})
        _eq(sd, want)
    assert restore_cache.stats["stores"] == h0["stores"] + 1
    assert restore_cache.stats["hits"] == h0["hits"] + 2
    # a new take at the same path: new metadata identity -> a new plan
    sd["a"].add_(1)
    Snapshot.take(path, {"sd": sd}, compression="hsz1")
    want = {k: v.clone() for k, v in sd.items()}
    for v in sd.values():
        v.zero_()
    Snapshot(path).restore({"sd": sd})
    _eq(sd, want)
    assert restore_cache.stats["stores"] == h0["stores"] + 2
    # a replaced leaf: no hit
    hits = restore_cache.stats["hits"]
    sd["b"] = torch.zeros(300, 7, device=gpu)
    Snapshot(path).restore({"sd": sd})
    _eq(sd, want)
    assert restore_cache.stats["hits"] == hits
    restore_cache.clear()


def test_read_object_with_budget_keeps_pinned_slots_within_it(gpu, tmp_path):
    """A budgeted read_object into an HBM tensor goes through the native job
    with pinned slots of at most half the budget."""
    from hipsnapshot.engine import native_restore
    from hipsnapshot.knobs import override_is_batching_disabled
    from hipsnapshot.ops import native

    big = torch.randn(64 << 20, device=gpu)  # 256 MiB
    path = str(tmp_path / "o")
    with override_is_batching_disabled(True):
        Snapshot.take(path, {"sd": StateDict(big=big)})
    native.pinned_trim()
    # (blocks held for the process's life, e.g. the slab-gap zero page, stay)
    cached0, used0 = native.pinned_stats()
    out = torch.zeros_like(big)
    native_restore.last_stats.clear()
    budget = 32 << 20
    Snapshot(path).read_object("0/sd/big", obj_out=out, memory_budget_bytes=budget)
    torch.cuda.synchronize()
    assert torch.equal(out, big)
    assert native_restore.last_stats.get("items", 0) > 0
    cached, used = native.pinned_stats()
    assert used == used0
    assert cached - cached0 <= budget // 2 + (4 << 20), (cached, cached0)


def test_native_restore_error_mid_job_then_clean_restore(gpu, tmp_path):
    """A corrupt blob among several fails the restore without hanging; the
    next restore of an intact snapshot (same process, same pools) is exact."""
    from hipsnapshot.knobs import override_is_batching_disabled
    from hipsnapshot.ops import codec, native

    g = torch.Generator(device=gpu).manual_seed(4)
    sd = StateDict(**{f"t{i}": (torch.randn(1 << 21, device=gpu, generator=g) * 0.02)
                      .to(torch.bfloat16) for i in range(8)})
    bad_path, good_path = str(tmp_path / "bad"), str(tmp_path / "good")
    with override_is_batching_disabled(True):
        Snapshot.take(bad_path, {"sd": sd}, compression="hsz1")
        Snapshot.take(good_path, {"sd": sd}, compression="hsz1")
    f = os.path.join(bad_path, "0", "sd", "t3")
    h = codec.parse_header(open(f, "rb").read())
    with open(f, "r+b") as fh:  # frame 1's mode byte
        fh.seek(h.offsets[1])
        fh.write(b"\x09")
    out = _zeros_like_state(sd)
    with override_is_batching_disabled(True), override_knob("RESTORE_SLOT_BYTES", str(1 << 20)), \
            pytest.raises(native.CorruptBlobError, match="t3"):
        Snapshot(bad_path).restore({"sd": out})
    torch.cuda.synchronize()
    out = _zeros_like_state(sd)
    with override_is_batching_disabled(True):
        Snapshot(good_path).restore({"sd": out})
    torch.cuda.synchronize()
    _eq(out, sd)


def test_native_and_python_reads_in_one_restore(gpu, tmp_path):
    """HBM tensors go through the native job while a host tensor and an
    object take the Python pipeline, in the same restore."""
    from hipsnapshot.engine import native_restore

    g = torch.Generator(device=gpu).manual_seed(6)
    src = {"gpu": (torch.randn(3 << 20, device=gpu, generator=g) * 0.02).to(torch.bfloat16),
           "cpu": torch.randn(1 << 20),
           "obj": {"step": 7, "name": "x"}}
    path = str(tmp_path / "m")
    Snapshot.take(path, {"sd": StateDict(**src)}, compression="hsz1")
    dst = StateDict(gpu=torch.zeros_like(src["gpu"]), cpu=torch.zeros(1 << 20), obj=None)
    native_restore.last_stats.clear()
    Snapshot(path).restore({"sd": dst})
    torch.cuda.synchronize()
    assert native_restore.last_stats.get("items", 0) >= 1
    assert torch.equal(dst["gpu"], src["gpu"]) and torch.equal(dst["cpu"], src["cpu"])
    assert dst["obj"] == src["obj"]


@pytest.mark.parametrize("compression", ["none", "hsz1"])
def test_restore_never_reads_bytes_an_earlier_restore_left(gpu, tmp_path, compression):
    """Every idle block of the restore's device pools and of the pinned host
    pool is overwritten between restores of the same snapshot: a job that
    read a byte it had not written (upload / decode / copy-table space, or a
    pinned slot) would only be right because the previous restore left the
    same bytes there (round-5 trim A/B: wrong bytes once another process got
    the freed HBM)."""
    from hipsnapshot.engine import native_restore
    from hipsnapshot.ops import native

    src = _state(gpu)
    path = str(tmp_path / "s")
    Snapshot.take(path, {"sd": src}, compression=compression)
    dev = torch.cuda.current_device()
    for i, byte in enumerate((0xA5, 0x00, 0xFF, 0x7F)):
        dst = _zeros_like_state(src)
        native_restore.last_stats.clear()
        Snapshot(path).restore({"sd": dst}, verify=(i % 2 == 1))
        torch.cuda.synchronize()
        assert native_restore.last_stats.get("items", 0) > 0
        _eq(dst, src)
        assert native.poison_idle_pools(dev, byte) > 0
    # budgeted reads: 1 MiB pinned slots, many pieces per blob
    for name in ("big", "w", "h"):
        for byte in (0x5A, 0xC3):
            out = torch.zeros_like(src[name])
            native.poison_idle_pools(dev, byte)
            Snapshot(path).read_object(f"0/sd/{name}", obj_out=out, memory_budget_bytes=2048)
            torch.cuda.synchronize()
            assert torch.equal(out, src[name]), (name, byte)


def test_resharded_restore_never_reads_stale_pool_bytes(gpu, tmp_path):
    from hipsnapshot.utils.test_utils import run_distributed

    run_distributed(_poison_reshard_worker, 2, str(tmp_path), timeout=600)


def _poison_reshard_worker(root):
    import torch.distributed as dist
    from torch.distributed.device_mesh import init_device_mesh
    from torch.distributed.tensor import DTensor, Shard

    from hipsnapshot.ops import native

    rank = dist.get_rank()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    mesh = init_device_mesh("cuda", (2,))  # both ranks on this GPU

    def dt(local, dim):
        return DTensor.from_local(local, mesh, [Shard(dim)], run_check=False)

    g = torch.Generator(device=dev).manual_seed(7)
    full = (torch.randn(512, 384, device=dev, generator=g) * 0.02).to(torch.bfloat16)
    want = full[:, rank * 192:(rank + 1) * 192]
    for comp in ("none", "hsz1"):
        path = os.path.join(root, comp)
        Snapshot.take(path, {"sd": StateDict(x=dt(full[rank * 256:(rank + 1) * 256].clone(), 0))},
                      compression=comp)
        for byte in (0xA5, 0xFF, 0x00):
            native.poison_idle_pools(0, byte)
            loc = torch.zeros(512, 192, device=dev, dtype=torch.bfloat16)
            Snapshot(path).restore({"sd": StateDict(x=dt(loc, 1))})
            torch.cuda.synchronize()
            assert torch.equal(loc, want), (comp, byte)
            out = torch.zeros(512, 384, device=dev, dtype=torch.bfloat16)
            native.poison_idle_pools(0, byte ^ 0x3C)
            Snapshot(path).read_object("0/sd/x", obj_out=out, memory_budget_bytes=2048)
            torch.cuda.synchronize()
            assert torch.equal(out, full), (comp, byte, "read_object")


def test_pools_trimmed_to_zero_four_processes_bitwise(gpu, tmp_path):
    """The round-5 failure: 4 processes restoring on one GPU with the restore
    pools freed after EVERY job (and ``release_restore_memory()`` between
    reads) got wrong bytes and hipErrorIllegalAddress faults: after freeing
    both uncached and plain hipMalloc'd blocks, the process's kernels used
    its next blocks through stale translations (profiles/r6/trim/).  The pools now allocate through the VMM hooks, whose
    freed addresses are never handed out again: every read is bitwise, with
    and without ``verify``, whole and in 2 KiB tiles."""
    import sys

    sys.path.insert(0, os.path.dirname(__file__))
    import test_dtensor_2d as T

    from hipsnapshot.utils.test_utils import run_distributed

    run_distributed(T._save_worker, 4, str(tmp_path), "cuda:0", timeout=600)
    run_distributed(_trim_zero_worker, 4, str(tmp_path), timeout=600)


def _trim_zero_worker(tmp):
    from hipsnapshot import release_restore_memory
    from hipsnapshot.knobs import override_tuning
    from hipsnapshot.ops import native

    ref = torch.load(f"{tmp}/ref.pt", weights_only=True)
    names = ("layers.0.attention.wq.weight", "layers.1.feed_forward.w2.weight",
             "tok_embeddings.weight")
    with override_tuning(restore_keep_bytes=0):
        for it in range(4):
            for name in names:
                for budget in (None, 2048):
                    out = torch.zeros_like(ref[f"m/{name}"]).to("cuda:0")
                    Snapshot(f"{tmp}/async").read_object(f"0/model/{name}", obj_out=out,
                                                         memory_budget_bytes=budget,
                                                         verify=bool(it % 2))
                    torch.cuda.synchronize()
                    assert torch.equal(out.cpu(), ref[f"m/{name}"]), (it, name, budget)
            release_restore_memory()
    assert native.require_gpu_lib().hsg_rt_vmm_retired_bytes() > 0  # the pools were freed


def test_vmm_blocks_survive_mixed_churn_across_processes(gpu, tmp_path):
    """The hook the pools allocate through, outside the engine: 4 processes
    allocate an uncached and a plain block, SDMA-upload a tagged pattern,
    copy it through both with the copy kernel, read it back and free both,
    300 times each.  With hipMalloc / hipExtMallocWithFlags the same loop
    returned wrong or foreign words in 117 of 1200 iterations (466 of 600 in
    one process); with the VMM blocks none (scripts/probes/pool_churn_mp.py,
    profiles/r6/trim/)."""
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = tmp_path / "churn.json"
    proc = subprocess.run([sys.executable, os.path.join(root, "scripts/probes/pool_churn_mp.py"),
                           "--mode", "both", "--alloc", "vmm", "--procs", "4", "--iters", "300",
                           "--out", str(out)], capture_output=True, text=True, timeout=300)
    assert proc.returncode == 0, proc.stderr[-2000:]
    res = json.load(open(out))
    assert res["errors"] == 0 and res["bad_iters"] == 0, json.dumps(res)[:2000]
    assert all(r["iters"] == 300 for r in res["ranks"])
