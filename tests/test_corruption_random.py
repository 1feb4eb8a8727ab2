"""Randomised storage corruption: after a take of a random state, one random
blob is damaged -- a flipped byte, truncation, deletion, appended garbage,
or zeroed bytes -- and then:

* ``verify_snapshot`` must report that blob (mismatched or missing);
* ``restore(verify=True)`` must raise, never return wrong tensors;
* a plain restore may raise or return (without checksums a flipped raw byte
  is undetectable, as in the reference), but it must not crash or hang --
  on the GPU, the native restore and the HSZ1 decoder must reject short or
  damaged blobs instead of faulting.
"""

import os
import random

import pytest
import torch

from hipsnapshot import Snapshot, StateDict
from hipsnapshot.verify import verify_snapshot

DAMAGE = ["flip", "truncate", "delete", "append", "zero"]


def _state(rng: random.Random, device: str) -> dict:
    out = {}
    for i in range(rng.randint(1, 5)):
        n = rng.choice([7, 1000, rng.randint(10_000, 600_000)])
        dtype = rng.choice([torch.float32, torch.bfloat16, torch.int64])
        t = (torch.randn(n) * 10).to(dtype)
        out[f"t{i}"] = t.to(device)
    return out


def _blobs(root: str):
    out = []
    for d, _dirs, files in os.walk(root):
        for f in files:
            p = os.path.join(d, f)
            rel = os.path.relpath(p, root)
            if rel.startswith(".snapshot") or os.path.getsize(p) == 0:
                continue
            out.append((rel, p))
    return sorted(out)


def _damage(rng: random.Random, p: str, how: str) -> None:
    size = os.path.getsize(p)
    if how == "delete":
        os.remove(p)
    elif how == "truncate":
        with open(p, "r+b") as f:
            f.truncate(rng.randrange(size))
    elif how == "append":
        with open(p, "ab") as f:
            f.write(os.urandom(rng.randint(1, 100)))
    else:
        with open(p, "r+b") as f:
            pos = rng.randrange(size)
            f.seek(pos)
            b = f.read(1)[0]
            f.seek(pos)
            if how == "flip":
                f.write(bytes([b ^ (1 << rng.randrange(8))]))
            else:  # zero a run
                f.write(bytes(min(size - pos, rng.randint(1, 4096))))


def _case(tmp_path, seed: int, device: str) -> None:
    rng = random.Random(seed)
    state = _state(rng, device)
    path = os.path.join(str(tmp_path), f"c{seed}")
    comp = rng.choice(["none", "hsz1", "hsz1+host"])
    Snapshot.take(path, {"sd": StateDict(**state)}, compression=comp)
    blobs = _blobs(path)
    rel, p = rng.choice(blobs)
    how = rng.choice(DAMAGE)
    before = open(p, "rb").read()
    _damage(rng, p, how)
    after = open(p, "rb").read() if os.path.exists(p) else None
    case = (seed, device, comp, rel, how)
    if after == before:  # e.g. zeroing bytes that were zero already
        return
    rep = verify_snapshot(path)
    assert not rep.ok, case
    assert any(rel in m or m in rel for m in rep.mismatched + rep.missing_blobs), (case, rep)

    def blank():
        return StateDict(**{k: torch.zeros_like(v) for k, v in state.items()})

    out = blank()
    with pytest.raises(Exception):
        Snapshot(path).restore({"sd": out}, verify=True)
    out = blank()
    try:
        Snapshot(path).restore({"sd": out})
    except Exception:  # noqa: BLE001 - a clean error is a fine answer
        pass
    if device != "cpu":
        torch.cuda.synchronize()  # the device is still healthy
        assert torch.equal(torch.ones(4, device=device).sum().cpu(), torch.tensor(4.0))


@pytest.mark.parametrize("seed", range(int(os.environ.get("HS_CORRUPT_SEEDS", "10"))))
def test_random_corruption_is_caught_cpu(tmp_path, seed):
    _case(tmp_path, seed, "cpu")


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(100, 100 + int(os.environ.get("HS_CORRUPT_SEEDS", "16"))))
def test_random_corruption_is_caught_gpu(tmp_path, gpu, seed):
    _case(tmp_path, seed, "cuda:0")
