"""On-disk format: manifest schema, flatten/inflate, dtype + byte encodings."""

from .flatten import decode_key, encode_key, flatten, inflate  # noqa: F401
from .manifest import (  # noqa: F401
    ChunkedTensorEntry,
    DictEntry,
    Entry,
    ListEntry,
    Manifest,
    ObjectEntry,
    OrderedDictEntry,
    PrimitiveEntry,
    Shard,
    ShardedTensorEntry,
    SnapshotMetadata,
    TensorEntry,
    entry_from_dict,
    is_container_entry,
    is_dict_entry,
    is_replicated,
    iter_tensor_entries,
)
from .serialization import (  # noqa: F401
    Serializer,
    dtype_to_element_size,
    dtype_to_string,
    string_to_dtype,
)
