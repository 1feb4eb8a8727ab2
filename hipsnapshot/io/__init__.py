"""Per-object I/O planning (tensor / chunked / sharded / object / primitive) + batching."""

from .preparer import get_storage_path, prepare_read, prepare_write  # noqa: F401
