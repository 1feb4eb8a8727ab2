"""Import-compatible entry point for code written against TorchSnapshot.

``import torchsnapshot`` resolves to hipsnapshot, and so do the reference's
module paths (``torchsnapshot.snapshot``, ``torchsnapshot.storage_plugin``,
``torchsnapshot.tricks.deepspeed``, ...; the table below).  Each alias is the
hipsnapshot module object itself -- no wrapper, no copy -- so
``mock.patch("torchsnapshot.storage_plugin.FSStoragePlugin", ...)`` and
``isinstance`` checks behave as they do against hipsnapshot.  Snapshots are
format-compatible both ways, HSZ1 / fp8 blobs aside.

Module layout of the reference: `/root/reference/torchsnapshot/`.
"""

from __future__ import annotations

import importlib
import importlib.abc
import importlib.util
import sys

# reference module path -> hipsnapshot module
ALIASES = {
    "snapshot": "hipsnapshot.snapshot",
    "stateful": "hipsnapshot.stateful",
    "state_dict": "hipsnapshot.stateful",
    "rng_state": "hipsnapshot.stateful",
    "version": "hipsnapshot.version",
    "knobs": "hipsnapshot.knobs",
    "manifest": "hipsnapshot.format.manifest",
    "flatten": "hipsnapshot.format.flatten",
    "serialization": "hipsnapshot.format.serialization",
    "io_types": "hipsnapshot.io_types",
    "io_preparer": "hipsnapshot.io.preparer",
    "io_preparers": "hipsnapshot.io",
    "io_preparers.tensor": "hipsnapshot.io.tensor",
    "io_preparers.chunked_tensor": "hipsnapshot.io.chunked",
    "io_preparers.sharded_tensor": "hipsnapshot.io.sharded",
    "io_preparers.object": "hipsnapshot.io.object",
    "batcher": "hipsnapshot.io.batcher",
    "partitioner": "hipsnapshot.parallel.partitioner",
    "manifest_ops": "hipsnapshot.parallel.elasticity",
    "pg_wrapper": "hipsnapshot.parallel.comm",
    "dist_store": "hipsnapshot.parallel.store",
    "scheduler": "hipsnapshot.engine.scheduler",
    "storage_plugin": "hipsnapshot.storage.registry",
    "storage_plugins": "hipsnapshot.storage",
    "storage_plugins.fs": "hipsnapshot.storage.fs",
    "storage_plugins.s3": "hipsnapshot.storage.s3",
    "storage_plugins.gcs": "hipsnapshot.storage.gcs",
    "memoryview_stream": "hipsnapshot.storage.memoryview_stream",
    "uvm_tensor": "hipsnapshot.ops.uvm",
    "rss_profiler": "hipsnapshot.utils.rss_profiler",
    "test_utils": "hipsnapshot.utils.test_utils",
    "tricks": "hipsnapshot.tricks",
    "tricks.deepspeed": "hipsnapshot.tricks.deepspeed",
}


class _AliasLoader(importlib.abc.Loader):
    def __init__(self, target: str) -> None:
        self.target = target

    def create_module(self, spec):
        return importlib.import_module(self.target)

    def exec_module(self, module) -> None:  # already executed as its real name
        pass


class _AliasFinder(importlib.abc.MetaPathFinder):
    def find_spec(self, fullname, path=None, target=None):
        if not fullname.startswith(__name__ + "."):
            return None
        target_name = ALIASES.get(fullname[len(__name__) + 1:])
        if target_name is None:
            return None
        return importlib.util.spec_from_loader(fullname, _AliasLoader(target_name))


def _warn_if_shadowing() -> None:
    """The hipsnapshot wheel ships this top-level ``torchsnapshot`` package;
    a real TorchSnapshot distribution installed alongside would overwrite (or
    be overwritten by) it.  Say so instead of failing in odd ways later."""
    import importlib.metadata as md
    import warnings

    for dist_name in ("torchsnapshot", "torchsnapshot-nightly"):
        try:
            md.distribution(dist_name)
        except md.PackageNotFoundError:
            continue
        warnings.warn(
            f"the '{dist_name}' distribution is installed next to hipsnapshot's torchsnapshot "
            "alias package; they share the top-level 'torchsnapshot' name. Uninstall one of "
            "them (hipsnapshot's alias maps the reference API onto hipsnapshot).",
            RuntimeWarning, stacklevel=3)


_warn_if_shadowing()

if not any(isinstance(f, _AliasFinder) for f in sys.meta_path):
    sys.meta_path.insert(0, _AliasFinder())

from hipsnapshot import (  # noqa: E402
    AppState,
    PendingSnapshot,
    RNGState,
    Snapshot,
    StateDict,
    Stateful,
    __version__,
)

__all__ = ["Snapshot", "PendingSnapshot", "Stateful", "StateDict", "RNGState", "AppState",
           "__version__"]
