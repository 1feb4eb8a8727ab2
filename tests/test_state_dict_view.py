"""snapshot._plain_state_dict: the iterative state_dict walk used on a take's
unblock path must return exactly what ``nn.Module.state_dict(keep_vars=True)``
returns (keys, order, tensor objects, ``_metadata``), run each pre hook once,
and step aside for anything it does not reproduce."""

import torch
import torch.nn as nn

from hipsnapshot.snapshot import _plain_state_dict, _state_dict_view


class _Block(nn.Module):
    def __init__(self):
        super().__init__()
        self.lin = nn.Linear(8, 8)
        self.bn = nn.BatchNorm1d(8)
        self.register_buffer("scratch", torch.zeros(2), persistent=False)
        self.register_buffer("kept", torch.ones(2))
        self.register_parameter("absent", None)


def _model():
    m = nn.Sequential(*[_Block() for _ in range(5)],
                      nn.ModuleDict({"x": nn.Linear(3, 3), "y": nn.Embedding(4, 2)}))
    m[3].lin.weight = m[1].lin.weight  # shared: listed under both names
    return m


def _same(a, b):
    assert list(a) == list(b)
    assert all(a[k] is b[k] for k in a)
    assert a._metadata == b._metadata


def test_matches_nn_module_state_dict():
    m = _model()
    _same(m.state_dict(keep_vars=True), _plain_state_dict(m))


def test_pre_hooks_run_once_in_module_order():
    m = _model()
    seen = []
    m[2].register_state_dict_pre_hook(lambda mod, prefix, kv: seen.append(("a", prefix, kv)))
    m[4].lin.register_state_dict_pre_hook(lambda mod, prefix, kv: seen.append(("b", prefix, kv)))
    ref = m.state_dict(keep_vars=True)
    expect, seen[:] = list(seen), []
    _same(ref, _plain_state_dict(m))
    assert seen == expect == [("a", "2.", True), ("b", "4.lin.", True)]


def test_pre_hook_that_swaps_a_parameter_is_seen():
    """FSDP2's pre hook re-points parameters at their sharded versions: the
    walk must read a module's parameters after its hooks ran."""
    m = _model()
    new = nn.Parameter(torch.full((8, 8), 3.0))

    def swap(mod, prefix, kv):
        mod.lin.weight = new

    m[0].register_state_dict_pre_hook(swap)
    assert _plain_state_dict(m)["0.lin.weight"] is new


def test_falls_back_for_what_it_does_not_reproduce():
    class Extra(nn.Linear):
        def get_extra_state(self):
            return {"k": 1}

    class Custom(nn.Linear):
        def _save_to_state_dict(self, destination, prefix, keep_vars):
            destination[prefix + "custom"] = torch.zeros(1)

    assert _plain_state_dict(nn.Sequential(Extra(2, 2))) is None
    assert _plain_state_dict(nn.Sequential(Custom(2, 2))) is None
    post = nn.Linear(2, 2)
    post.register_state_dict_post_hook(lambda *a: None)
    assert _plain_state_dict(nn.Sequential(post)) is None
    # a module that stops qualifying after the first check is caught in the walk
    m = _model()
    assert _plain_state_dict(m) is not None
    m[1].add_module("late", Extra(2, 2))
    assert _plain_state_dict(m) is None
    sd = _state_dict_view(m)  # the full state_dict, extra state included
    assert "1.late._extra_state" in sd


def test_state_dict_view_detaches_plain_parameters():
    m = _model()
    sd = _state_dict_view(m)
    assert not sd["0.lin.weight"].requires_grad
    assert sd["0.lin.weight"].data_ptr() == m[0].lin.weight.data_ptr()


def test_optimizer_state_materialized_without_moving_params_or_hooks():
    from hipsnapshot.snapshot import _materialize_optimizer_state

    m = nn.Linear(4, 4)
    opt = torch.optim.AdamW(m.parameters(), lr=0.1, weight_decay=0.5)
    seen = []
    opt.register_step_post_hook(lambda *a: seen.append(1))
    w = m.weight.detach().clone()
    assert _materialize_optimizer_state(opt)
    assert len(opt.state) == 2 and not seen
    assert torch.equal(m.weight, w) and m.weight.grad is None
    assert opt.param_groups[0]["lr"] == 0.1
    # a parameter holding a gradient: left alone
    m2 = nn.Linear(2, 2)
    m2.weight.grad = torch.ones_like(m2.weight)
    assert not _materialize_optimizer_state(torch.optim.SGD(m2.parameters(), lr=1.0))
