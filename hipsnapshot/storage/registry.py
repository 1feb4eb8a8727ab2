"""URL -> storage plugin routing.

Reference: `/root/reference/torchsnapshot/storage_plugin.py:18-78`.  ``proto://path``
selects the backend (``fs`` when no protocol is given); built-ins are ``fs``,
``s3``, ``gs`` and ``memory`` (an in-process object store used by tests and
benchmarks); third-party plugins register a factory
``(path, storage_options) -> StoragePlugin`` under the entry-point group
``storage_plugins`` (same group name as the reference, so existing plugin
packages are discovered), or programmatically via :func:`register_storage_plugin`.
"""

from __future__ import annotations

import asyncio
from typing import Any, Callable, Dict, Optional

from ..io_types import StoragePlugin
from . import fs as _fs
from .fs import FSStoragePlugin

# the reference's tests swap the FS plugin with
# mock.patch("torchsnapshot.storage_plugin.FSStoragePlugin", ...); ours patch
# hipsnapshot.storage.fs.FSStoragePlugin -- either replacement is honoured
_FS_PLUGIN = FSStoragePlugin

Factory = Callable[[str, Optional[Dict[str, Any]]], StoragePlugin]
_REGISTRY: Dict[str, Factory] = {}


def register_storage_plugin(protocol: str, factory: Factory) -> None:
    _REGISTRY[protocol] = factory


def _builtin(protocol: str, path: str, storage_options) -> Optional[StoragePlugin]:
    if protocol == "fs":
        cls = FSStoragePlugin if FSStoragePlugin is not _FS_PLUGIN else _fs.FSStoragePlugin
        return cls(root=path, storage_options=storage_options)
    if protocol == "s3":
        from .s3 import S3StoragePlugin

        return S3StoragePlugin(root=path, storage_options=storage_options)
    if protocol in ("gs", "gcs"):
        from .gcs import GCSStoragePlugin

        return GCSStoragePlugin(root=path, storage_options=storage_options)
    if protocol == "memory":
        from .memory import MemoryStoragePlugin

        return MemoryStoragePlugin(root=path, storage_options=storage_options)
    return None


def split_url(url_path: str):
    if "://" in url_path:
        protocol, path = url_path.split("://", 1)
        if not protocol:
            raise RuntimeError(f"Invalid url: {url_path}")
        return protocol, path
    return "fs", url_path


def url_to_storage_plugin(url_path: str,
                          storage_options: Optional[Dict[str, Any]] = None) -> StoragePlugin:
    protocol, path = split_url(url_path)
    if protocol in _REGISTRY:
        return _REGISTRY[protocol](path, storage_options)
    plugin = _builtin(protocol, path, storage_options)
    if plugin is not None:
        return plugin
    try:
        from importlib.metadata import entry_points

        eps = entry_points()
        group = eps.select(group="storage_plugins") if hasattr(eps, "select") \
            else eps.get("storage_plugins", [])
        for ep in group:
            if ep.name == protocol:
                return ep.load()(path, storage_options)
    except Exception:  # pragma: no cover
        pass
    raise RuntimeError(f"Unsupported protocol: {protocol}.")


def url_to_storage_plugin_in_event_loop(url_path: str, event_loop: asyncio.AbstractEventLoop,
                                        storage_options: Optional[Dict[str, Any]] = None
                                        ) -> StoragePlugin:
    async def _make() -> StoragePlugin:
        return url_to_storage_plugin(url_path, storage_options)

    return event_loop.run_until_complete(_make())
