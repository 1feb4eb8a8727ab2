"""CPU-side pieces of the native restore: job sizing under a memory budget,
and that reads stay on the Python pipeline without a GPU."""

from hipsnapshot.engine import native_restore
from hipsnapshot.knobs import override_knob


def test_sizing_defaults_and_budget():
    slot, first, n = native_restore.sizing(None)
    assert slot == 128 << 20 and first == 16 << 20 and n == 6
    # a 100 MiB read budget: the pinned slots take at most half of it
    slot, first, n = native_restore.sizing(100 << 20)
    assert slot * n <= 50 << 20 and n >= 2 and first <= slot
    assert n == 6 and slot >= 4 << 20  # a deep pipeline of small slots, not 2 big ones
    # tiny budgets still get two 1 MiB slots
    slot, first, n = native_restore.sizing(1 << 20)
    assert (slot, n) == (1 << 20, 2) and first == 1 << 20
    with override_knob("RESTORE_SLOTS", "3"), override_knob("RESTORE_SLOT_BYTES", str(8 << 20)):
        assert native_restore.sizing(None) == (8 << 20, 8 << 20, 3)


def test_split_without_gpu_keeps_every_read_on_python(tmp_path):
    from hipsnapshot.io_types import ReadReq
    from hipsnapshot.storage.fs import FSStoragePlugin

    reqs = [ReadReq(path="a", buffer_consumer=None), ReadReq(path="b", buffer_consumer=None)]
    jobs, py = native_restore.split(reqs, FSStoragePlugin(str(tmp_path)))
    assert jobs == {} and py == reqs


def test_drain_booster_reaches_running_and_later_jobs():
    """PendingSnapshot.wait() boosts the drain jobs of its own take: those
    running, and one attached after the boost."""
    from hipsnapshot.engine.native_drain import Booster

    class Job:
        def __init__(self):
            self.boosted = 0

        def boost(self):
            self.boosted += 1

    b = Booster()
    a = Job()
    b.attach(a)
    assert a.boosted == 0
    b.boost()
    assert a.boosted == 1
    late = Job()
    b.attach(late)
    assert late.boosted == 1
    b.detach(a)
    b.detach(late)
    other = Booster()
    c = Job()
    other.attach(c)
    assert c.boosted == 0  # another take's drain keeps its parked writers


def test_prewarm_skips_without_gpu_and_codec_detection():
    """prewarm_for is a no-op without HBM destinations / GPU; _has_codec sees
    codecs of nested shard entries."""
    import torch

    from hipsnapshot.engine import native_restore
    from hipsnapshot.format.manifest import Shard, ShardedTensorEntry, TensorEntry

    native_restore.prewarm_for([torch.zeros(4)], [], None)  # CPU leaves: nothing starts
    assert native_restore._prewarm is None
    plain = TensorEntry("a", "torch_save", "torch.float32", [4], False)
    coded = TensorEntry("b", "buffer_protocol", "torch.bfloat16", [4], False,
                        codec={"name": "hsz1"})
    assert not native_restore._has_codec(plain)
    assert native_restore._has_codec(coded)
    assert native_restore._has_codec(ShardedTensorEntry([Shard([0], [4], coded)]))
    assert not native_restore._has_codec(ShardedTensorEntry([Shard([0], [4], plain)]))
