"""Randomised UVM (managed-memory) snapshots on the GPU: managed tables with
pages in host DRAM or in HBM, beside plain HBM tensors; random dtypes and
sizes, sync or async takes (async: CPU capture behind the stream gate, or
the HBM freeze), random capture threads / overlap, compression; the trainer
updates every table right after ``async_take`` returns.  Each snapshot must
hold the pre-update values; restores go into managed targets (either
residency) and into plain tensors, bitwise.  TorchRec's UVM tables are the
case (`/root/reference/torchsnapshot/uvm_tensor.py`).
"""

import os
import random

import pytest
import torch

from hipsnapshot import Snapshot, StateDict
from hipsnapshot.knobs import override_tuning

pytestmark = pytest.mark.gpu


def _state(rng: random.Random, dev: torch.device):
    from hipsnapshot.ops import uvm

    out = {}
    g = torch.Generator(device=dev).manual_seed(rng.randrange(1 << 30))
    for i in range(rng.randint(1, 5)):
        rows = rng.choice([1, 7, 1000, rng.randint(1, 1 << 18)])
        dim = rng.choice([1, 16, 64])
        dtype = rng.choice([torch.float32, torch.bfloat16, torch.int64])
        kind = rng.choice(["host", "device", "plain"])
        src = (torch.randn(rows, dim, device=dev, generator=g) * 100).to(dtype)
        if kind == "plain":
            t = src
        else:
            t = uvm.new_managed_tensor([rows, dim], dtype, dev.index or 0)
            t.copy_(src)
            uvm.place(t, kind)
        out[f"{kind}{i}"] = t
    torch.cuda.synchronize()
    return out


def _target(v: torch.Tensor, kind: str, dev):
    from hipsnapshot.ops import uvm

    if kind == "plain":
        return torch.zeros_like(v)
    t = uvm.new_managed_tensor(list(v.shape), v.dtype, dev.index or 0)
    t.zero_()
    uvm.place(t, kind)
    return t


def _case(tmp_path, seed: int, dev) -> None:
    rng = random.Random(seed)
    state = _state(rng, dev)
    tuning = dict(uvm_async_capture=rng.random() < 0.8,
                  uvm_capture_threads=rng.choice([1, 4, 32]),
                  uvm_capture_overlap=rng.random() < 0.5)
    comp = rng.choice(["none", "hsz1"])
    use_async = rng.random() < 0.7
    case = (seed, tuning, comp, use_async, {k: tuple(v.shape) for k, v in state.items()})
    path = os.path.join(str(tmp_path), f"u{seed}")
    ref = {k: v.clone() for k, v in state.items()}
    with override_tuning(**tuning):
        app = {"sd": StateDict(**state)}
        if use_async:
            pending = Snapshot.async_take(path, app, compression=comp)
            for v in state.values():  # the trainer's next step
                v.add_(1)
            pending.wait()
        else:
            Snapshot.take(path, app, compression=comp)
    torch.cuda.synchronize()
    for k, v in state.items():
        if use_async:
            assert torch.equal(v, ref[k] + 1), (case, k)
    kinds = [rng.choice(["host", "device", "plain"]) for _ in state]
    out = StateDict(**{k: _target(v, kd, dev) for (k, v), kd in zip(ref.items(), kinds)})
    Snapshot(path).restore({"sd": out}, verify=rng.random() < 0.5)
    torch.cuda.synchronize()
    for k, v in ref.items():
        assert torch.equal(out[k], v), (case, k, kinds)


@pytest.mark.parametrize("seed", range(int(os.environ.get("HS_UVM_SEEDS", "8"))))
def test_random_uvm_snapshots(tmp_path, gpu, seed):
    _case(tmp_path, seed, gpu)
