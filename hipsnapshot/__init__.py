"""hipsnapshot: distributed checkpointing for PyTorch on AMD Instinct MI355X.

Public API (same surface as TorchSnapshot, reference `torchsnapshot/__init__.py:10-41`):
``Snapshot``, ``PendingSnapshot``, ``Stateful``, ``StateDict``, ``RNGState``,
``__version__``.
"""

import sys as _sys

import torch as _torch  # noqa: F401  (load torch's HIP runtime before our .so)

from .engine.hbm_staging import release_hbm_arena
from .engine.memory import held as memory_held
from .engine.memory import release_idle as release_snapshot_memory
from .engine.native_restore import release_restore_memory
from .snapshot import PendingSnapshot, Snapshot
from .stateful import AppState, RNGState, StateDict, Stateful
from .version import __hipsnapshot_version__, __version__


def _is_notebook() -> bool:
    try:
        from IPython import get_ipython  # type: ignore

        shell = get_ipython()
        return shell is not None and ("Terminal" not in type(shell).__name__)
    except Exception:
        return False


if _is_notebook():  # pragma: no cover - Jupyter/Colab nest their own loop
    try:
        import nest_asyncio  # type: ignore

        nest_asyncio.apply()
    except Exception:
        pass

__all__ = [
    "Snapshot",
    "PendingSnapshot",
    "Stateful",
    "StateDict",
    "RNGState",
    "AppState",
    "release_hbm_arena",
    "release_restore_memory",
    "release_snapshot_memory",
    "memory_held",
    "__version__",
    "__hipsnapshot_version__",
]
