"""Stateful protocol and the two built-in statefuls.

* ``Stateful`` / ``AppState`` -- reference `stateful.py:13-23`.
* ``StateDict`` -- a ``UserDict`` that is Stateful (reference `state_dict.py:13-41`).
* ``RNGState`` -- reference `rng_state.py:13-38` captures the CPU generator only;
  ours also captures every visible HIP device generator (``cuda`` in torch
  naming) when ``include_device=True`` (default), so a resumed MI355X job
  replays dropout masks exactly.  CPU-only snapshots stay reference-compatible
  (the extra key is simply absent).
"""

from __future__ import annotations

from collections import UserDict
from typing import Any, Dict, Protocol, runtime_checkable

import torch


@runtime_checkable
class Stateful(Protocol):
    def state_dict(self) -> Dict[str, Any]:
        ...

    def load_state_dict(self, state_dict: Dict[str, Any]) -> None:
        ...


AppState = Dict[str, Stateful]


class StateDict(UserDict):
    """A dict that can be put in ``app_state`` directly (counters, progress...)."""

    def state_dict(self) -> Dict[str, Any]:
        return self.data

    def load_state_dict(self, state_dict: Dict[str, Any]) -> None:
        self.data.update(state_dict)


class RNGState:
    """Snapshot-able RNG state.

    ``Snapshot`` guarantees the RNG state is identical right after ``take`` and
    right after ``restore`` of the same snapshot (it is captured first on take
    and restored last on restore).
    """

    def __init__(self, include_device: bool = True) -> None:
        self.include_device = include_device

    def state_dict(self) -> Dict[str, Any]:
        sd: Dict[str, Any] = {"rng_state": torch.get_rng_state()}
        if self.include_device and torch.cuda.is_available() and torch.cuda.is_initialized():
            for i in range(torch.cuda.device_count()):
                sd[f"hip_rng_state_{i}"] = torch.cuda.get_rng_state(i)
        return sd

    def load_state_dict(self, state_dict: Dict[str, Any]) -> None:
        torch.set_rng_state(state_dict["rng_state"])
        if self.include_device and torch.cuda.is_available():
            for k, v in state_dict.items():
                if k.startswith("hip_rng_state_"):
                    idx = int(k.rsplit("_", 1)[1])
                    if idx < torch.cuda.device_count():
                        torch.cuda.set_rng_state(v, idx)
