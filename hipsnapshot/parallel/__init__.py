"""Distributed planning: comm facade (RCCL/gloo), store barrier, partitioner, elasticity."""

from .comm import Comm, PGWrapper  # noqa: F401
from .elasticity import get_manifest_for_rank, handle_sharded_tensor_elasticity  # noqa: F401
from .partitioner import consolidate_replicated_entries, partition_write_reqs  # noqa: F401
from .store import LinearBarrier, create_store, get_or_create_store  # noqa: F401
