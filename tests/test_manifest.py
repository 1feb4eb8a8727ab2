"""Manifest schema: JSON round trip, YAML compatibility, per-rank views, format conformance."""

import json
import math

import pytest
import yaml

from hipsnapshot.format.manifest import (
    ChunkedTensorEntry,
    DictEntry,
    ListEntry,
    ObjectEntry,
    OrderedDictEntry,
    PrimitiveEntry,
    Shard,
    ShardedTensorEntry,
    SnapshotMetadata,
    TensorEntry,
)
from hipsnapshot.parallel.elasticity import get_manifest_for_rank, handle_sharded_tensor_elasticity


def _te(loc, rep=False, br=None):
    return TensorEntry(location=loc, serializer="buffer_protocol", dtype="torch.float32",
                       shape=[2, 3], replicated=rep, byte_range=br)


def _manifest():
    return {
        "0/foo": DictEntry(keys=["bar", "baz", "qux", "quux", "sharded", "chunked", "obj"]),
        "0/foo/bar": _te("0/foo/bar"),
        "0/foo/baz": _te("replicated/foo/baz", rep=True),
        "0/foo/qux": PrimitiveEntry.from_object(3.25),
        "0/foo/quux": ListEntry(),
        "0/foo/quux/0": PrimitiveEntry.from_object(b"\x00\x01"),
        "0/foo/sharded": ShardedTensorEntry(shards=[Shard([0, 0], [1, 3], _te("sharded/x_0_0"))]),
        "0/foo/chunked": ChunkedTensorEntry(
            dtype="torch.float32", shape=[4, 3],
            chunks=[Shard([0, 0], [2, 3], _te("0/foo/chunked_0_0", br=[0, 24])),
                    Shard([2, 0], [2, 3], _te("0/foo/chunked_2_0"))], replicated=False),
        "0/foo/obj": ObjectEntry(location="0/foo/obj", serializer="torch_save",
                                 obj_type="builtins.set", replicated=False),
        "1/foo": OrderedDictEntry(keys=["bar", "sharded"]),
        "1/foo/bar": _te("1/foo/bar"),
        "1/foo/sharded": ShardedTensorEntry(shards=[Shard([1, 0], [1, 3], _te("sharded/x_1_0"))]),
    }


def test_json_roundtrip_and_yaml_compat():
    md = SnapshotMetadata(version="0.1.0", world_size=2, manifest=_manifest())
    text = md.to_json()
    d = json.loads(text)
    # exact on-disk field layout
    assert list(d) == ["version", "world_size", "manifest"]
    assert list(d["manifest"]["0/foo/bar"]) == ["type", "location", "serializer", "dtype", "shape",
                                               "replicated", "byte_range"]
    assert list(d["manifest"]["0/foo/qux"]) == ["type", "serialized_value", "replicated",
                                               "readable"]
    assert SnapshotMetadata.from_json(text) == md
    # a YAML-dumped metadata (older writers) parses too
    assert SnapshotMetadata.from_yaml(yaml.dump(d)) == md


def test_primitive_encodings():
    for v in [0, -7, "s/%x", True, False, b"\xff\x00", 1.0 / 3.0, math.inf, -0.0]:
        e = PrimitiveEntry.from_object(v)
        back = PrimitiveEntry.from_dict(json.loads(json.dumps(e.to_dict()))).get_value()
        assert type(back) is type(v) and (back == v or (v != v and back != back))
        if isinstance(v, float):
            assert e.readable == str(v)
    # reference float encoding: base64 of the packed C double
    assert PrimitiveEntry.from_object(1.5).serialized_value == "AAAAAAAA+D8="


def test_manifest_for_existing_and_new_ranks():
    md = SnapshotMetadata(version="0.1.0", world_size=2, manifest=_manifest())
    m0, merged = get_manifest_for_rank(md, 0)
    assert "foo/baz" in m0 and "foo/bar" in m0
    assert len(merged["foo/sharded"].shards) == 2
    assert len(m0["foo/sharded"].shards) == 2
    m1, _ = get_manifest_for_rank(md, 1)
    assert "foo/baz" in m1  # replicated entries visible to every rank
    assert m1["foo/bar"].location == "1/foo/bar"
    assert len(m1["foo/sharded"].shards) == 2
    for rank in (2, 3):  # upscaled ranks see replicated + containers only
        mn, _ = get_manifest_for_rank(md, rank)
        assert set(mn) == {"foo", "foo/baz", "foo/quux"}
        assert mn["foo"].keys == ["baz", "quux"]


def test_sharded_elasticity_add_and_remove():
    md = SnapshotMetadata(version="0.1.0", world_size=2, manifest=_manifest())
    mn, merged = get_manifest_for_rank(md, 3)
    handle_sharded_tensor_elasticity(mn, merged, ["foo/sharded"])
    assert "foo/sharded" in mn and "sharded" in mn["foo"].keys
    m0, merged = get_manifest_for_rank(md, 0)
    handle_sharded_tensor_elasticity(m0, merged, [])
    assert "foo/sharded" not in m0


def test_old_layout_replicated_under_every_rank():
    man = _manifest()
    man["1/foo/baz"] = _te("replicated/foo/baz", rep=True)
    md = SnapshotMetadata(version="0.1.0", world_size=2, manifest=man)
    m1, _ = get_manifest_for_rank(md, 1)
    assert m1["foo/baz"].replicated


def test_unknown_entry_type_rejected():
    with pytest.raises(ValueError):
        SnapshotMetadata.from_json(json.dumps(
            {"version": "0.1.0", "world_size": 1, "manifest": {"0/x": {"type": "Bogus"}}}))


def test_fragment_joined_metadata_matches_object_encoding():
    """take() joins per-rank pre-encoded JSON fragments; the result must equal
    encoding the consolidated manifest objects."""
    import json

    from hipsnapshot.format.manifest import (LazySnapshotMetadata, SnapshotMetadata, entry_json,
                                             metadata_json_from_parts)
    from hipsnapshot.snapshot import Snapshot

    class OneRank:
        def get_world_size(self):
            return 1

        def get_rank(self):
            return 0

        def all_gather_object(self, out, obj):
            out[0] = obj

    man = {
        "m/w": TensorEntry("0/m/w", "buffer_protocol", "torch.float32", [3, 4], False),
        "m/r": TensorEntry("replicated/m/r", "buffer_protocol", "torch.bfloat16", [8], True,
                           codec={"name": "hsz1", "w": 2, "frame_bytes": 256, "blob_bytes": 16}),
        "m/s": PrimitiveEntry.from_object("a/b\"c", replicated=False),
    }
    md = Snapshot._gather_metadata(dict(man), OneRank())
    assert isinstance(md, LazySnapshotMetadata)
    ref = SnapshotMetadata(version=md.version, world_size=1,
                           manifest={"0/m/w": man["m/w"], "0/m/s": man["m/s"],
                                     "0/m/r": man["m/r"]})
    assert json.loads(md.to_json()) == ref.to_dict()
    assert list(md.manifest) == ["0/m/w", "0/m/s", "0/m/r"]
    assert md.manifest["0/m/r"].codec["name"] == "hsz1"
    assert metadata_json_from_parts("0.1.0", 2, []) == \
        '{"version":"0.1.0","world_size":2,"manifest":{}}'
    assert json.loads(entry_json(man["m/w"])) == man["m/w"].to_dict()


def test_manifest_for_rank_copies_are_independent():
    """Restore mutates the per-rank view (elasticity adds/drops entries and
    edits dict keys); the cached split must not see those edits."""
    from hipsnapshot.format.manifest import DictEntry, Shard, ShardedTensorEntry

    def te(loc):
        return TensorEntry(loc, "buffer_protocol", "torch.float32", [2, 2], False)

    man = {
        "0/sd": DictEntry(keys=["a", "w"]),
        "0/sd/a": te("0/sd/a"),
        "0/sd/w": ShardedTensorEntry([Shard([0, 0], [1, 2], te("sharded/sd/w_0_0"))]),
        "1/sd": DictEntry(keys=["a", "w"]),
        "1/sd/a": te("1/sd/a"),
        "1/sd/w": ShardedTensorEntry([Shard([1, 0], [1, 2], te("sharded/sd/w_1_0"))]),
    }
    md = SnapshotMetadata(version="0.1.0", world_size=2, manifest=man)
    local, merged = get_manifest_for_rank(md, 0)
    assert len(local["sd/w"].shards) == 2
    local["sd"].keys.remove("a")
    del local["sd/a"]
    merged.clear()
    again, merged2 = get_manifest_for_rank(md, 0)
    assert again["sd"].keys == ["a", "w"] and "sd/a" in again and "sd/w" in merged2
    assert man["0/sd"].keys == ["a", "w"]
