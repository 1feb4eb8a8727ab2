"""DeepSpeed ZeRO-3 integration trick (demonstration, like the reference's).

Reference: `/root/reference/torchsnapshot/tricks/deepspeed.py:19-103`.  Patches a
``DeepSpeedEngine`` so ``_save_zero_checkpoint`` persists the (already
partitioned, per-rank) ZeRO optimizer state with ``Snapshot.async_take`` --
training resumes after the HBM freeze instead of waiting for storage -- and
``_load_zero_checkpoint`` restores it through ``Zero3StateAdapter``.

DeepSpeed is not installed in this environment, so the module only
duck-types the engine/optimizer (attributes used: ``optimizer``, ``config``,
``global_rank``, ``_copy_recovery_script``, ``zero_load_from_fp32_weights``,
``optimizer._rigid_load_state_dict``, ``optimizer.persistent_parameters``);
``require_zero3=True`` additionally checks the optimizer class name.
"""

from __future__ import annotations

import logging
from types import MethodType
from typing import Any, Dict, Optional

from ..snapshot import PendingSnapshot, Snapshot
from ..stateful import StateDict
from ..version import __version__

logger = logging.getLogger(__name__)


class Zero3StateAdapter:
    """Exposes a ZeRO-3 optimizer through ``state_dict`` / ``load_state_dict``."""

    def __init__(self, optimizer: Any, load_optimizer_states: bool = True,
                 load_from_fp32_weights: bool = False) -> None:
        self.optimizer = optimizer
        self.load_optimizer_state = load_optimizer_states
        self.load_from_fp32_weights = load_from_fp32_weights

    def state_dict(self) -> Dict[str, Any]:
        return self.optimizer.state_dict()

    def load_state_dict(self, state_dict: Dict[str, Any]) -> None:
        self.optimizer._rigid_load_state_dict(state_dict=state_dict,
                                              load_optimizer_states=self.load_optimizer_state)
        persistent = getattr(self.optimizer, "persistent_parameters", None) or []
        if len(persistent) > 0:
            persistent[0].partition(persistent)
            persistent[0].all_gather(persistent)


def _save_zero_checkpoint(self, save_path: str, tag: str) -> None:
    app_state = {
        "optimizer": self.optimizer,
        "objects": StateDict(ds_config=_plain(getattr(self, "config", None)),
                             hipsnapshot_version=__version__),
    }
    self._hipsnapshot_pending = Snapshot.async_take(path=save_path, app_state=app_state)
    if getattr(self, "global_rank", 0) == 0 and hasattr(self, "_copy_recovery_script"):
        self._copy_recovery_script(save_path)


def _load_zero_checkpoint(self, load_dir: str, tag: str,
                          load_optimizer_states: bool = True) -> bool:
    pending: Optional[PendingSnapshot] = getattr(self, "_hipsnapshot_pending", None)
    if pending is not None:
        pending.wait()
    lf = getattr(self, "zero_load_from_fp32_weights", None)
    app_state = {"optimizer": Zero3StateAdapter(
        self.optimizer, load_optimizer_states=load_optimizer_states,
        load_from_fp32_weights=lf() if callable(lf) else False)}
    Snapshot(path=load_dir).restore(app_state=app_state)
    return True


def _plain(cfg: Any) -> Any:
    """DeepSpeed configs are objects; persist a plain dict/str view."""
    if cfg is None or isinstance(cfg, (dict, str, int, float, bool)):
        return cfg
    for attr in ("_param_dict", "__dict__"):
        d = getattr(cfg, attr, None)
        if isinstance(d, dict):
            return {k: v for k, v in d.items() if isinstance(v, (dict, str, int, float, bool,
                                                                  list, type(None)))}
    return str(cfg)


def patch_engine_to_use_hipsnapshot(engine: Any, require_zero3: bool = True) -> None:
    """Route a DeepSpeed engine's ZeRO checkpoint save/load through hipsnapshot.

    WARNING: like the reference, a demonstration integration, not an official
    DeepSpeed checkpoint engine.
    """
    if require_zero3 and type(engine.optimizer).__name__ != "DeepSpeedZeroOptimizer_Stage3":
        raise RuntimeError(
            "patch_engine_to_use_hipsnapshot only supports DeepSpeedZeroOptimizer_Stage3.")
    engine._save_zero_checkpoint = MethodType(_save_zero_checkpoint, engine)
    engine._load_zero_checkpoint = MethodType(_load_zero_checkpoint, engine)


# reference-compatible name
patch_engine_to_use_torchsnapshot = patch_engine_to_use_hipsnapshot
