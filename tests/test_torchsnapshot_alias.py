"""``import torchsnapshot`` works for code written against the reference."""

import asyncio
from unittest import mock

import pytest
import torch


def test_reference_module_paths_resolve_to_hipsnapshot():
    import hipsnapshot
    import torchsnapshot
    from torchsnapshot import RNGState, Snapshot, StateDict, Stateful  # noqa: F401
    from torchsnapshot.dist_store import LinearBarrier, get_or_create_store  # noqa: F401
    from torchsnapshot.flatten import flatten, inflate  # noqa: F401
    from torchsnapshot.io_preparer import prepare_read, prepare_write  # noqa: F401
    from torchsnapshot.io_preparers.chunked_tensor import ChunkedTensorIOPreparer  # noqa: F401
    from torchsnapshot.io_preparers.sharded_tensor import ShardedTensorIOPreparer  # noqa: F401
    from torchsnapshot.io_preparers.tensor import TensorIOPreparer, tensor_copy  # noqa: F401
    from torchsnapshot.manifest import SnapshotMetadata, TensorEntry  # noqa: F401
    from torchsnapshot.manifest_ops import get_manifest_for_rank  # noqa: F401
    from torchsnapshot.memoryview_stream import MemoryviewStream  # noqa: F401
    from torchsnapshot.pg_wrapper import PGWrapper  # noqa: F401
    from torchsnapshot.rss_profiler import measure_rss_deltas  # noqa: F401
    from torchsnapshot.scheduler import get_process_memory_budget_bytes  # noqa: F401
    from torchsnapshot.serialization import Serializer  # noqa: F401
    from torchsnapshot.storage_plugin import url_to_storage_plugin  # noqa: F401
    from torchsnapshot.storage_plugins.fs import FSStoragePlugin  # noqa: F401
    from torchsnapshot.test_utils import assert_state_dict_eq, rand_tensor  # noqa: F401
    from torchsnapshot.tricks.deepspeed import patch_engine_to_use_torchsnapshot  # noqa: F401
    from torchsnapshot.uvm_tensor import is_uvm_tensor  # noqa: F401

    assert torchsnapshot.Snapshot is hipsnapshot.Snapshot
    import hipsnapshot.snapshot as real
    import torchsnapshot.snapshot as alias

    assert alias is real
    with pytest.raises(ModuleNotFoundError):
        import torchsnapshot.does_not_exist  # noqa: F401


def test_reference_style_take_restore_and_plugin_patch(tmp_path):
    import torchsnapshot
    from torchsnapshot.storage_plugins.fs import FSStoragePlugin

    model = torch.nn.Linear(32, 8)
    progress = torchsnapshot.StateDict(current_epoch=3)
    app_state = {"model": model, "progress": progress, "rng": torchsnapshot.RNGState()}
    snap = torchsnapshot.Snapshot.take(path=str(tmp_path / "ok"), app_state=app_state)
    w = model.weight.detach().clone()
    with torch.no_grad():
        model.weight.zero_()
    progress["current_epoch"] = 0
    snap.restore(app_state=app_state)
    assert torch.equal(model.weight, w) and progress["current_epoch"] == 3

    class Faulty(FSStoragePlugin):
        async def write(self, write_io):
            await asyncio.sleep(0)
            raise OSError("injected through the reference's patch point")

    with mock.patch("torchsnapshot.storage_plugin.FSStoragePlugin", Faulty):
        with pytest.raises(OSError, match="reference's patch point"):
            torchsnapshot.Snapshot.take(path=str(tmp_path / "bad"), app_state=app_state)
