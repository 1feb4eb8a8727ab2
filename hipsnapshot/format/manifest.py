"""Manifest entries and snapshot metadata (the on-disk schema).

The schema is a tagged union keyed by ``"type"`` and is kept JSON-identical to
the reference (`/root/reference/torchsnapshot/manifest.py:28-314`) so that a
``.snapshot_metadata`` written by either implementation is readable by the
other:

* ``Tensor``        {location, serializer, dtype, shape, replicated, byte_range}
* ``ShardedTensor`` {shards: [{offsets, sizes, tensor: Tensor}]}
* ``ChunkedTensor`` {dtype, shape, chunks: [Shard], replicated}
* ``object``        {location, serializer, obj_type, replicated}
* ``list`` / ``dict`` {keys} / ``OrderedDict`` {keys}
* primitives ``int|str|bool|bytes|float`` {serialized_value, replicated, readable}

Metadata is written as JSON (fast) and read with ``json`` first, falling back
to YAML ``SafeLoader`` for metadata produced by YAML dumpers (JSON is a subset
of YAML, reference `manifest.py:283-314`).

hipsnapshot extensions: a ``Tensor`` entry may carry an optional ``quant``
object (only present for the opt-in fp8 serializer) and an optional ``codec``
object (opt-in lossless HSZ1 compression of the blob it lives in:
``{"name": "hsz1", "w": 2, "frame_bytes": F, "blob_bytes": L}``, its
``byte_range`` staying in logical bytes); both are omitted from the JSON when
absent so ordinary snapshots are byte-compatible.
"""

from __future__ import annotations

import base64
import json
import struct
from dataclasses import dataclass, field
from typing import Any, ClassVar, Dict, List, Optional, Tuple, Union

Key = Union[str, int]


@dataclass
class Entry:
    type: str

    def to_dict(self) -> Dict[str, Any]:  # pragma: no cover - overridden
        return {"type": self.type}


@dataclass(init=False)
class TensorEntry(Entry):
    location: str
    serializer: str
    dtype: str
    shape: List[int]
    replicated: bool
    byte_range: Optional[List[int]]
    quant: Optional[Dict[str, Any]] = None
    codec: Optional[Dict[str, Any]] = None

    def __init__(
        self,
        location: str,
        serializer: str,
        dtype: str,
        shape: List[int],
        replicated: bool,
        byte_range: Optional[List[int]] = None,
        quant: Optional[Dict[str, Any]] = None,
        codec: Optional[Dict[str, Any]] = None,
    ) -> None:
        self.type = "Tensor"
        self.location = location
        self.serializer = serializer
        self.dtype = dtype
        self.shape = list(shape)
        self.replicated = replicated
        self.byte_range = list(byte_range) if byte_range is not None else None
        self.quant = quant
        self.codec = codec

    @property
    def byte_range_tuple(self) -> Optional[Tuple[int, int]]:
        if self.byte_range is None:
            return None
        return (int(self.byte_range[0]), int(self.byte_range[1]))

    def to_dict(self) -> Dict[str, Any]:
        d = {
            "type": self.type,
            "location": self.location,
            "serializer": self.serializer,
            "dtype": self.dtype,
            "shape": list(self.shape),
            "replicated": self.replicated,
            "byte_range": list(self.byte_range) if self.byte_range is not None else None,
        }
        if self.quant is not None:
            d["quant"] = self.quant
        if self.codec is not None:
            d["codec"] = self.codec
        return d

    @classmethod
    def from_dict(cls, d: Dict[str, Any]) -> "TensorEntry":
        return cls(
            location=d["location"],
            serializer=d["serializer"],
            dtype=d["dtype"],
            shape=d["shape"],
            replicated=d.get("replicated", False),
            byte_range=d.get("byte_range"),
            quant=d.get("quant"),
            codec=d.get("codec"),
        )


@dataclass
class Shard:
    offsets: List[int]
    sizes: List[int]
    tensor: TensorEntry

    def to_dict(self) -> Dict[str, Any]:
        return {"offsets": list(self.offsets), "sizes": list(self.sizes),
                "tensor": self.tensor.to_dict()}

    @classmethod
    def from_dict(cls, d: Dict[str, Any]) -> "Shard":
        return cls(offsets=list(d["offsets"]), sizes=list(d["sizes"]),
                   tensor=TensorEntry.from_dict(d["tensor"]))


@dataclass(init=False)
class ShardedTensorEntry(Entry):
    shards: List[Shard]

    def __init__(self, shards: List[Shard]) -> None:
        self.type = "ShardedTensor"
        self.shards = shards

    def to_dict(self) -> Dict[str, Any]:
        return {"type": self.type, "shards": [s.to_dict() for s in self.shards]}

    @classmethod
    def from_dict(cls, d: Dict[str, Any]) -> "ShardedTensorEntry":
        return cls(shards=[Shard.from_dict(s) for s in d["shards"]])

    def global_shape(self) -> List[int]:
        if not self.shards:
            return []
        shape = [0] * len(self.shards[0].sizes)
        for s in self.shards:
            for i, (o, z) in enumerate(zip(s.offsets, s.sizes)):
                shape[i] = max(shape[i], o + z)
        return shape


@dataclass(init=False)
class ChunkedTensorEntry(Entry):
    dtype: str
    shape: List[int]
    chunks: List[Shard]
    replicated: bool

    def __init__(self, dtype: str, shape: List[int], chunks: List[Shard],
                 replicated: bool) -> None:
        self.type = "ChunkedTensor"
        self.dtype = dtype
        self.shape = list(shape)
        self.chunks = chunks
        self.replicated = replicated

    def to_dict(self) -> Dict[str, Any]:
        return {"type": self.type, "dtype": self.dtype, "shape": list(self.shape),
                "chunks": [c.to_dict() for c in self.chunks],
                "replicated": self.replicated}

    @classmethod
    def from_dict(cls, d: Dict[str, Any]) -> "ChunkedTensorEntry":
        return cls(dtype=d["dtype"], shape=d["shape"],
                   chunks=[Shard.from_dict(c) for c in d["chunks"]],
                   replicated=d.get("replicated", False))


@dataclass(init=False)
class ObjectEntry(Entry):
    location: str
    serializer: str
    obj_type: str
    replicated: bool

    def __init__(self, location: str, serializer: str, obj_type: str,
                 replicated: bool) -> None:
        self.type = "object"
        self.location = location
        self.serializer = serializer
        self.obj_type = obj_type
        self.replicated = replicated

    def to_dict(self) -> Dict[str, Any]:
        return {"type": self.type, "location": self.location,
                "serializer": self.serializer, "obj_type": self.obj_type,
                "replicated": self.replicated}

    @classmethod
    def from_dict(cls, d: Dict[str, Any]) -> "ObjectEntry":
        return cls(location=d["location"], serializer=d["serializer"],
                   obj_type=d["obj_type"], replicated=d.get("replicated", False))


@dataclass(init=False)
class ListEntry(Entry):
    def __init__(self) -> None:
        self.type = "list"

    def to_dict(self) -> Dict[str, Any]:
        return {"type": self.type}

    @classmethod
    def from_dict(cls, d: Dict[str, Any]) -> "ListEntry":
        return cls()


@dataclass(init=False)
class DictEntry(Entry):
    keys: List[Key]

    def __init__(self, keys: List[Key]) -> None:
        self.type = "dict"
        self.keys = list(keys)

    def to_dict(self) -> Dict[str, Any]:
        return {"type": self.type, "keys": list(self.keys)}

    @classmethod
    def from_dict(cls, d: Dict[str, Any]) -> "DictEntry":
        return cls(keys=d["keys"])


@dataclass(init=False)
class OrderedDictEntry(Entry):
    keys: List[Key]

    def __init__(self, keys: List[Key]) -> None:
        self.type = "OrderedDict"
        self.keys = list(keys)

    def to_dict(self) -> Dict[str, Any]:
        return {"type": self.type, "keys": list(self.keys)}

    @classmethod
    def from_dict(cls, d: Dict[str, Any]) -> "OrderedDictEntry":
        return cls(keys=d["keys"])


PRIMITIVE_TYPES = ("int", "str", "bool", "bytes", "float")


@dataclass(init=False)
class PrimitiveEntry(Entry):
    """A primitive stored inline in the metadata (no blob).

    Encodings (reference `manifest.py:179-270`): int/str/bool as ``str(x)``,
    bytes as base64, float as base64 of the packed C double (bit exact) with a
    human ``readable`` copy.
    """

    supported_types: ClassVar[Tuple[str, ...]] = PRIMITIVE_TYPES
    serialized_value: str
    replicated: bool
    readable: Optional[str]

    def __init__(self, type: str, serialized_value: str, replicated: bool = False,
                 readable: Optional[str] = None) -> None:
        if type not in PRIMITIVE_TYPES:
            raise TypeError(f"Unsupported primitive obj of type {type}")
        self.type = type
        self.serialized_value = serialized_value
        self.replicated = replicated
        self.readable = readable

    def get_value(self) -> Union[int, str, bool, bytes, float]:
        t, v = self.type, self.serialized_value
        if t == "int":
            return int(v)
        if t == "str":
            return v
        if t == "bool":
            if v not in ("True", "False"):
                raise RuntimeError(f"Unexpected serialized_value for bool type: {v}")
            return v == "True"
        if t == "bytes":
            return base64.b64decode(v.encode("utf-8"))
        if t == "float":
            return struct.unpack("d", base64.b64decode(v.encode("utf-8")))[0]
        raise ValueError(f"Unable to get deserialized value for {v}")

    @staticmethod
    def serialize(type_name: str, obj: Any) -> str:
        if type_name in ("int", "str", "bool"):
            return str(obj)
        if type_name == "bytes":
            return base64.b64encode(obj).decode("utf-8")
        if type_name == "float":
            return base64.b64encode(struct.pack("d", float(obj))).decode("utf-8")
        raise TypeError(f"Unsupported primitive obj of type {type_name}")

    @classmethod
    def from_object(cls, obj: Any, replicated: bool = False) -> "PrimitiveEntry":
        type_name = type(obj).__name__
        if type_name not in PRIMITIVE_TYPES:
            raise TypeError(f"Unsupported primitive obj of type {type_name}")
        return cls(type_name, cls.serialize(type_name, obj), replicated,
                   str(obj) if type_name == "float" else None)

    def to_dict(self) -> Dict[str, Any]:
        return {"type": self.type, "serialized_value": self.serialized_value,
                "replicated": self.replicated, "readable": self.readable}

    @classmethod
    def from_dict(cls, d: Dict[str, Any]) -> "PrimitiveEntry":
        return cls(d["type"], d["serialized_value"], d.get("replicated", False),
                   d.get("readable"))


Manifest = Dict[str, Entry]

_ENTRY_TYPES = {
    "Tensor": TensorEntry,
    "ShardedTensor": ShardedTensorEntry,
    "ChunkedTensor": ChunkedTensorEntry,
    "object": ObjectEntry,
    "list": ListEntry,
    "dict": DictEntry,
    "OrderedDict": OrderedDictEntry,
}


def entry_from_dict(d: Dict[str, Any]) -> Entry:
    t = d["type"]
    if t in PRIMITIVE_TYPES:
        return PrimitiveEntry.from_dict(d)
    cls = _ENTRY_TYPES.get(t)
    if cls is None:
        raise ValueError(f"Unrecognized entry type {t!r}")
    return cls.from_dict(d)


@dataclass
class SnapshotMetadata:
    version: str
    world_size: int
    manifest: Manifest = field(default_factory=dict)

    def to_dict(self) -> Dict[str, Any]:
        return {"version": self.version, "world_size": self.world_size,
                "manifest": {k: v.to_dict() for k, v in self.manifest.items()}}

    def to_json(self) -> str:
        # Compact separators keep json on its C encoder: ~10x faster than the
        # reference's indent=2 (pure-Python encoder), which matters for the
        # merged manifest of an 8-rank FSDP job.  Any JSON/YAML reader parses it.
        pre = self.__dict__.get("_json_async")
        if pre is not None:
            thread, box = pre
            thread.join()
            if "json" in box:
                return box["json"]
        return json.dumps(self.to_dict(), sort_keys=False, separators=(",", ":"))

    def serialize_in_background(self) -> None:
        """Start encoding the JSON now (the commit needs it only after all
        blobs are written): takes the merged-manifest encoding of an 8-rank
        job off rank 0's critical path.  The manifest must not change after
        this call; ``to_json`` joins the thread."""
        import threading

        box: Dict[str, str] = {}

        def run() -> None:
            try:
                box["json"] = json.dumps(self.to_dict(), sort_keys=False,
                                         separators=(",", ":"))
            except Exception:  # noqa: BLE001 - to_json falls back to inline encoding
                pass

        t = threading.Thread(target=run, name="hipsnapshot-metadata-json", daemon=True)
        t.start()
        self.__dict__["_json_async"] = (t, box)

    # Reference name (metadata is JSON, which is valid YAML).
    def to_yaml(self) -> str:
        return self.to_json()

    @classmethod
    def from_dict(cls, d: Dict[str, Any]) -> "SnapshotMetadata":
        manifest = {path: entry_from_dict(e) for path, e in d["manifest"].items()}
        return cls(version=str(d["version"]), world_size=int(d["world_size"]),
                   manifest=manifest)

    @classmethod
    def from_json(cls, text: str) -> "SnapshotMetadata":
        from ..utils.tracing import paused_gc

        with paused_gc():
            return cls._from_json(text)

    @classmethod
    def _from_json(cls, text: str) -> "SnapshotMetadata":
        try:
            d = json.loads(text)
        except json.JSONDecodeError:
            import yaml

            loader = getattr(yaml, "CSafeLoader", yaml.SafeLoader)
            d = yaml.load(text, Loader=loader)
        return cls.from_dict(d)

    from_yaml = from_json


def is_container_entry(entry: Entry) -> bool:
    return isinstance(entry, (ListEntry, DictEntry, OrderedDictEntry))


def is_dict_entry(entry: Entry) -> bool:
    return isinstance(entry, (DictEntry, OrderedDictEntry))


def is_replicated(entry: Entry) -> bool:
    return bool(getattr(entry, "replicated", False))


def iter_tensor_entries(entry: Entry):
    """Yield every ``TensorEntry`` (blob descriptor) inside ``entry``."""
    if isinstance(entry, TensorEntry):
        yield entry
    elif isinstance(entry, ChunkedTensorEntry):
        for c in entry.chunks:
            yield c.tensor
    elif isinstance(entry, ShardedTensorEntry):
        for s in entry.shards:
            yield s.tensor


class LazySnapshotMetadata(SnapshotMetadata):
    """Metadata assembled as JSON text (per-rank pre-encoded fragments joined
    on the committing rank); entry objects are only materialised if someone
    reads ``manifest``.  Keeps the 8-rank manifest encode/decode off the
    take's critical path."""

    def __init__(self, text: str, version: str, world_size: int) -> None:
        self.version = version
        self.world_size = world_size
        self._text: Optional[str] = text
        self._manifest: Optional[Manifest] = None

    @property
    def manifest(self) -> Manifest:  # type: ignore[override]
        if self._manifest is None:
            self._manifest = SnapshotMetadata.from_json(self._text).manifest
        return self._manifest

    @manifest.setter
    def manifest(self, value: Manifest) -> None:
        self._manifest = value
        self._text = None

    def to_json(self) -> str:
        if self._text is not None and self._manifest is None:
            return self._text
        return SnapshotMetadata.to_json(self)


_COMPACT = json.JSONEncoder(separators=(",", ":"))  # one encoder, not one per entry


def entry_json(entry: Entry) -> str:
    return _COMPACT.encode(entry.to_dict())


def metadata_json_from_parts(version: str, world_size: int, parts: List[str]) -> str:
    """``parts`` = ``'"<rank>/<path>":<entry json>'`` strings in manifest order."""
    return ('{"version":' + json.dumps(version) + ',"world_size":' + str(int(world_size))
            + ',"manifest":{' + ",".join(parts) + "}}")
