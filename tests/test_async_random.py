"""Randomised training loops around ``async_take``: every step mutates the
state in place; on random steps an ``async_take`` (or a blocking take) is
started without waiting for the ones still draining, with random options
(compression, HBM freeze vs host fallback, checksums on or off per take).  At the end every
snapshot must hold exactly the state of its own step -- the consistency
guarantee of `/root/reference/torchsnapshot/snapshot.py` ``async_take``
("changes to app_state after this returns do not affect the snapshot") --
and pass ``verify``.
"""

import os
import random

import pytest
import torch

from hipsnapshot import Snapshot, StateDict
from hipsnapshot.knobs import override_knob


def _state(rng: random.Random, device: str) -> dict:
    big = 2_000_000 if device != "cpu" else 300_000
    out = {}
    for i in range(rng.randint(3, 7)):
        n = rng.choice([1, 17, 4096, big, rng.randint(1, big)])
        dtype = rng.choice([torch.float32, torch.bfloat16, torch.float16])
        out[f"t{i}"] = torch.randn(n, device=device).to(dtype)
    out["m"] = torch.randn(rng.randint(2, 300), rng.randint(2, 300), device=device)
    return out


def _mutate(rng: random.Random, state: dict, step: int) -> None:
    for k, t in state.items():
        op = rng.randrange(3)
        if op == 0:
            t.add_(1.0 + step)
        elif op == 1:
            t.mul_(-0.5)
        else:
            t.index_fill_(0, torch.tensor([0], device=t.device), float(step))


def _loop(tmp_path, seed: int, device: str, steps: int = 10) -> None:
    rng = random.Random(seed)
    torch.manual_seed(seed)
    state = _state(rng, device)
    taken = []  # (path, refs, how)
    pending = []
    _steps(rng, state, steps, tmp_path, device, taken, pending)
    for _path, p in pending:
        p.wait()
    _check(taken)


def _steps(rng, state, steps, tmp_path, device, taken, pending) -> None:
    for step in range(steps):
        _mutate(rng, state, step)
        if rng.random() < 0.6:
            path = os.path.join(str(tmp_path), f"step_{step}")
            refs = {k: v.clone() for k, v in state.items()}
            comp = rng.choice(["none", "hsz1"])
            host_fallback = device != "cpu" and rng.random() < 0.3
            # CHECKSUM changes between takes while earlier ones still drain:
            # each async take drains with the knobs of its own call
            checksum = rng.choice(["0", "1"])
            how = (step, comp, host_fallback, checksum)
            with override_knob("HBM_STAGING_RESERVE_BYTES",
                               str(1 << 50) if host_fallback else "0"), \
                    override_knob("CHECKSUM", checksum):
                app = {"sd": StateDict(step=step, **state)}
                if rng.random() < 0.2:
                    Snapshot.take(path, app, compression=comp)
                else:
                    pending.append((path, Snapshot.async_take(path, app, compression=comp)))
            taken.append((path, refs, how))
            if pending and rng.random() < 0.3:
                pending.pop(rng.randrange(len(pending)))[1].wait()
        # read back a committed snapshot while later async takes still drain
        busy = {pp for pp, p in pending if not p.done()}
        done = [t for t in taken if t[0] not in busy]
        if done and rng.random() < 0.25:
            path, refs, how = rng.choice(done)
            out = StateDict(step=-1, **{k: torch.zeros_like(v) for k, v in refs.items()})
            Snapshot(path).restore({"sd": out})
            assert out["step"] == how[0] and all(torch.equal(out[k], v) for k, v in refs.items()), \
                ("restore during drains", how)


def _check(taken) -> None:
    from hipsnapshot.verify import verify_snapshot

    for path, refs, how in taken:
        out = StateDict(step=-1, **{k: torch.zeros_like(v) for k, v in refs.items()})
        Snapshot(path).restore({"sd": out})
        assert out["step"] == how[0], how
        for k, v in refs.items():
            assert torch.equal(out[k], v), (how, k)
        if how[3] == "1":
            assert verify_snapshot(path).ok, how


@pytest.mark.parametrize("seed", range(3))
def test_random_async_training_loop_cpu(tmp_path, seed):
    _loop(tmp_path, seed, "cpu")


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(100, 100 + int(os.environ.get("HS_ASYNC_GPU_SEEDS", "6"))))
def test_random_async_training_loop_gpu(tmp_path, gpu, seed):
    _loop(tmp_path, seed, "cuda:0")


def test_async_take_drains_with_the_knobs_of_its_call(tmp_path, monkeypatch):
    """The environment changes after ``async_take`` returns but before its
    drain writes (the commit thread is held back 0.3 s here): the drain still
    uses the call's knobs -- its checksums are written (``knobs.pinned``).
    The random loops above flip CHECKSUM between overlapping takes."""
    import time

    from hipsnapshot.snapshot import PendingSnapshot
    from hipsnapshot.verify import verify_snapshot

    orig = PendingSnapshot._complete_snapshot

    def late(self, *a, **kw):
        time.sleep(0.3)
        return orig(self, *a, **kw)

    monkeypatch.setattr(PendingSnapshot, "_complete_snapshot", late)
    sd = StateDict(w=torch.randn(1000, 100), step=3)
    with override_knob("CHECKSUM", "1"):
        pending = Snapshot.async_take(str(tmp_path / "a"), {"sd": sd})
    with override_knob("CHECKSUM", "0"):  # while the drain has not started
        pending.wait()
    rep = verify_snapshot(str(tmp_path / "a"))
    assert rep.has_checksums and rep.ok, rep
