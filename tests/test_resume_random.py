"""Resume equivalence, randomised: a random MLP with a random optimizer
(SGD with momentum / nesterov, Adam, AdamW, RMSprop, Adagrad; optionally a
LR scheduler) trains a few steps, is snapshotted together with the RNG
state, and keeps training K more steps -- the reference trajectory.  A FRESH
model + optimizer (+ scheduler) restored from the snapshot must then train
the same K steps to bit-identical weights and losses (dropout draws from the
restored RNG).  This is what a checkpoint is for; the reference checks it on
fixed cases (`/root/reference/tests/test_snapshot.py`, `test_rng_state.py`).
"""

import os
import random

import pytest
import torch
import torch.nn as nn

from hipsnapshot import RNGState, Snapshot

OPTIMS = [
    lambda p, r: torch.optim.SGD(p, lr=0.05, momentum=r.choice([0.0, 0.9]),
                                 nesterov=False, weight_decay=r.choice([0.0, 1e-4])),
    lambda p, r: torch.optim.SGD(p, lr=0.05, momentum=0.9, nesterov=True),
    lambda p, r: torch.optim.Adam(p, lr=1e-3, amsgrad=r.random() < 0.5),
    lambda p, r: torch.optim.AdamW(p, lr=1e-3, weight_decay=0.01),
    lambda p, r: torch.optim.RMSprop(p, lr=1e-3, momentum=r.choice([0.0, 0.5])),
    lambda p, r: torch.optim.Adagrad(p, lr=0.01),
]


def _model(rng: random.Random, device: str) -> nn.Module:
    dims = [rng.randint(2, 48) for _ in range(rng.randint(2, 4))]
    layers = []
    for a, b in zip(dims, dims[1:]):
        layers += [nn.Linear(a, b), rng.choice([nn.ReLU(), nn.Tanh(), nn.GELU()])]
        if rng.random() < 0.4:
            layers.append(nn.Dropout(0.2))
        if rng.random() < 0.3:
            layers.append(nn.LayerNorm(b))
    return nn.Sequential(*layers).to(device)


def _build(seed: int, device: str):
    rng = random.Random(seed)
    torch.manual_seed(seed)
    model = _model(rng, device)
    opt = rng.choice(OPTIMS)(model.parameters(), rng)
    sched = torch.optim.lr_scheduler.StepLR(opt, step_size=2, gamma=0.5) \
        if rng.random() < 0.5 else None
    batch = rng.randint(1, 16)
    return model, opt, sched, batch, model[0].in_features


def _step(model, opt, sched, batch, din, device) -> float:
    x = torch.randn(batch, din, device=device)  # from the (restored) RNG
    loss = model(x).pow(2).mean()
    opt.zero_grad(set_to_none=True)
    loss.backward()
    opt.step()
    if sched is not None:
        sched.step()
    return float(loss.item())


def _app(model, opt, sched):
    app = {"model": model, "optim": opt, "rng": RNGState()}
    if sched is not None:
        app["sched"] = sched
    return app


def _resume_case(tmp_path, seed: int, device: str) -> None:
    rng = random.Random(seed * 7 + 1)
    warm, k = rng.randint(1, 4), rng.randint(1, 4)
    model, opt, sched, batch, din = _build(seed, device)
    model.train()
    for _ in range(warm):
        _step(model, opt, sched, batch, din, device)
    path = os.path.join(str(tmp_path), f"r{seed}")
    comp = rng.choice(["none", "hsz1"])
    if rng.random() < 0.5:
        Snapshot.async_take(path, _app(model, opt, sched), compression=comp).wait()
    else:
        Snapshot.take(path, _app(model, opt, sched), compression=comp)
    ref_losses = [_step(model, opt, sched, batch, din, device) for _ in range(k)]
    ref_state = {n: p.detach().clone() for n, p in model.state_dict().items()}

    # a fresh process's view: new model (other init), new optimizer / scheduler
    model2, opt2, sched2, _b, _d = _build(seed, device)  # same architecture
    with torch.no_grad():
        for p in model2.parameters():
            p.add_(1.0)  # anything but the snapshot's values
    torch.manual_seed(seed + 999)  # and another RNG position
    Snapshot(path).restore(_app(model2, opt2, sched2))
    model2.train()
    losses = [_step(model2, opt2, sched2, batch, din, device) for _ in range(k)]
    case = (seed, device, type(opt).__name__, sched is not None, comp, warm, k)
    assert losses == ref_losses, case
    for n, v in model2.state_dict().items():
        assert torch.equal(v, ref_state[n]), (case, n)


@pytest.mark.parametrize("seed", range(int(os.environ.get("HS_RESUME_SEEDS", "4"))))
def test_random_resume_is_bit_identical_cpu(tmp_path, seed):
    _resume_case(tmp_path, seed, "cpu")


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(100, 100 + int(os.environ.get("HS_RESUME_SEEDS", "10"))))
def test_random_resume_is_bit_identical_gpu(tmp_path, gpu, seed):
    _resume_case(tmp_path, seed, "cuda:0")
