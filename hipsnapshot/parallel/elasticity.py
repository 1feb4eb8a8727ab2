"""Per-rank manifest views and world-size elasticity on restore.

Reference: `/root/reference/torchsnapshot/manifest_ops.py:24-216`.

* ``get_manifest_for_rank(metadata, rank)``: the entries a rank restores --
  its own per-rank entries, every replicated entry (stored under rank 0, or
  under every rank in the older layout), and sharded entries MERGED across all
  saving ranks (so any rank can reshard from any saved shard).  A rank >= the
  saved world size (upscaling) gets replicated + container entries only.
* ``handle_sharded_tensor_elasticity``: when all sharded entries sit at the
  root of their state dict, add sharded entries the target requests but the
  rank did not save, and drop the ones it does not request.

The rank split / shard merge is computed once per metadata object and cached
(reference re-derived and deep-copied it per stateful, Appendix C #9).
"""

from __future__ import annotations

import copy
from collections import defaultdict
from typing import Dict, List, Tuple

from ..format.manifest import (
    Entry,
    Manifest,
    ShardedTensorEntry,
    SnapshotMetadata,
    is_container_entry,
    is_dict_entry,
    is_replicated,
)


def _rank_split(metadata: SnapshotMetadata) -> Tuple[List[Dict[str, Entry]],
                                                       Dict[str, ShardedTensorEntry]]:
    cached = getattr(metadata, "_hs_rank_split", None)
    if cached is not None and cached[0] is metadata.manifest and cached[1] == len(metadata.manifest):
        return cached[2], cached[3]
    per_rank: List[Dict[str, Entry]] = [{} for _ in range(metadata.world_size)]
    for path, entry in metadata.manifest.items():
        rank_str, _, logical = path.partition("/")
        per_rank[int(rank_str)][logical] = entry
    groups: Dict[str, List[ShardedTensorEntry]] = defaultdict(list)
    for m in per_rank:
        for logical, e in m.items():
            if isinstance(e, ShardedTensorEntry):
                groups[logical].append(e)
    merged = {logical: ShardedTensorEntry(
        shards=sorted((s for e in g for s in e.shards), key=lambda s: s.offsets))
        for logical, g in groups.items()}
    try:
        metadata._hs_rank_split = (metadata.manifest, len(metadata.manifest), per_rank, merged)
    except AttributeError:  # pragma: no cover
        pass
    return per_rank, merged


def _fresh(entries: Dict[str, Entry]) -> Dict[str, Entry]:
    """A copy the restore path may mutate: new dict, new container entries
    (their ``keys`` lists are edited by the elasticity helpers); leaf entries
    are never mutated and are shared with the cached split (a deep copy of an
    8-rank FSDP manifest cost ~100 ms per restore)."""
    out = {}
    for logical, e in entries.items():
        if is_dict_entry(e):
            e = copy.copy(e)
            e.keys = list(e.keys)
        out[logical] = e
    return out


def get_manifest_for_rank(metadata: SnapshotMetadata, rank: int
                          ) -> Tuple[Manifest, Dict[str, ShardedTensorEntry]]:
    per_rank, merged = _rank_split(metadata)
    merged = dict(merged)
    if rank < metadata.world_size:
        local = _fresh(per_rank[rank])
        for logical, e in per_rank[0].items():
            if is_replicated(e):
                local[logical] = e
        for logical, e in list(local.items()):
            if isinstance(e, ShardedTensorEntry):
                local[logical] = merged[logical]
        return local, merged
    local = _fresh(per_rank[0])
    for logical in list(local):
        e = local.get(logical)
        if e is None or is_container_entry(e) or is_replicated(e):
            continue
        _remove_entry(local, logical)
    return local, merged


def handle_sharded_tensor_elasticity(manifest: Manifest,
                                     merged_sd_entries: Dict[str, ShardedTensorEntry],
                                     tensor_requests: List[str]) -> None:
    if not all(len(p.split("/")) == 2 for p in merged_sd_entries):
        return
    requests = [r for r in tensor_requests if r in merged_sd_entries]
    for logical in requests:
        if logical not in manifest:
            manifest[logical] = merged_sd_entries[logical]
            parent, _, key = logical.rpartition("/")
            pe = manifest.get(parent)
            if pe is not None and is_dict_entry(pe) and key not in pe.keys:
                pe.keys.append(key)
    req_set = set(requests)
    for logical in list(manifest):
        if isinstance(manifest[logical], ShardedTensorEntry) and logical not in req_set:
            del manifest[logical]


def _remove_entry(manifest: Manifest, logical_path: str) -> None:
    if logical_path not in manifest:
        return
    del manifest[logical_path]
    parent, sep, key = logical_path.rpartition("/")
    if not sep or not parent:
        return
    pe = manifest.get(parent)
    if pe is not None and is_dict_entry(pe):
        if key in pe.keys:
            pe.keys.remove(key)
        else:
            try:
                pe.keys.remove(int(key))
            except (ValueError, KeyError):
                pass
