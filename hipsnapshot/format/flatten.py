"""Reversible flattening of nested state dicts into ``{logical_path: leaf}``.

Same path grammar as the reference (`/root/reference/torchsnapshot/flatten.py:18-224`):

* a path is ``<prefix>/<k1>/<k2>/...``; each user key is escaped ``%``->``%25``
  then ``/``->``%2F`` so that ``/`` only ever denotes hierarchy;
* ``list`` recurses with decimal indices, ``dict``/``OrderedDict`` recurse when
  every key is ``str``/``int`` and their string forms are unique -- otherwise
  the dict is stored as an opaque leaf;
* containers get a manifest entry (``ListEntry``/``DictEntry``/``OrderedDictEntry``
  with the ORIGINAL keys, so int keys survive), leaves go to ``flattened``.

The implementation is iterative (explicit stack) so deeply nested optimizer
states do not hit the recursion limit.
"""

from __future__ import annotations

from collections import OrderedDict
from typing import Any, Dict, List, Tuple
from urllib.parse import unquote

from .manifest import DictEntry, Entry, ListEntry, Manifest, OrderedDictEntry


def encode_key(s: str) -> str:
    if "%" in s or "/" in s:
        return s.replace("%", "%25").replace("/", "%2F")
    return s  # (the common key: nothing to escape)


def decode_key(s: str) -> str:
    return unquote(s)


# reference-compatible private aliases
_encode = encode_key
_decode = decode_key


def _flattenable_dict(d: Dict[Any, Any]) -> bool:
    keys = list(d.keys())
    if not all(isinstance(k, (str, int)) for k in keys):
        return False
    return len({str(k) for k in keys}) == len(keys)


def flatten(obj: Any, prefix: str) -> Tuple[Manifest, Dict[str, Any]]:
    """Flatten ``obj`` under ``prefix`` -> (container manifest, leaves)."""
    manifest: Manifest = {}
    flattened: Dict[str, Any] = {}
    stack: List[Tuple[str, Any]] = [(encode_key(prefix), obj)]
    while stack:
        path, node = stack.pop()
        t = type(node)
        if t is list:
            manifest[path] = ListEntry()
            for idx in range(len(node) - 1, -1, -1):
                stack.append((f"{path}/{idx}", node[idx]))
        elif (t is dict or t is OrderedDict) and _flattenable_dict(node):
            keys = list(node.keys())
            manifest[path] = DictEntry(keys=keys) if t is dict else OrderedDictEntry(keys=keys)
            for k in reversed(keys):
                stack.append((f"{path}/{encode_key(str(k))}", node[k]))
        else:
            flattened[path] = node
    # Keep insertion order deterministic and parent-before-child (matches the
    # recursive definition): sort containers by DFS discovery already holds
    # for the stack walk above since children are pushed in reverse.
    return manifest, flattened


def _container_for(entry: Entry) -> Any:
    if isinstance(entry, ListEntry):
        return []
    if isinstance(entry, OrderedDictEntry):
        return OrderedDict.fromkeys(entry.keys)
    if isinstance(entry, DictEntry):
        return dict.fromkeys(entry.keys)
    raise RuntimeError(f"Unrecognized container entry type: {type(entry)} ({entry.type}).")


def inflate(manifest: Manifest, flattened: Dict[str, Any], prefix: str) -> Any:
    """Inverse of :func:`flatten`.

    Only keys present both in a dict entry's ``keys`` and among the supplied
    children survive, so callers can drop leaves by removing them from both.
    """
    root = encode_key(prefix)
    manifest = {k: v for k, v in manifest.items() if k.split("/", 1)[0] == root}
    flattened = {k: v for k, v in flattened.items() if k.split("/", 1)[0] == root}
    if root in flattened:
        return flattened[root]
    if root not in manifest:
        raise AssertionError(
            f"{root} is absent in both manifest and flattened.\n"
            f"manifest: {manifest}\nflattened: {flattened}")

    containers = {path: _container_for(e) for path, e in manifest.items()}
    children: Dict[str, Dict[str, Any]] = {}
    for source in (containers, flattened):
        for path, obj in source.items():
            if path == root:
                continue
            parent, sep, key = path.rpartition("/")
            if not sep:
                raise AssertionError(f"Invalid path: {path}")
            children.setdefault(parent, {})[key] = obj

    for path, vals in children.items():
        container = containers.get(path)
        if isinstance(container, list):
            container.extend(v for _, v in sorted(vals.items(), key=lambda kv: int(kv[0])))
        elif isinstance(container, dict):
            # flatten() names a child by str(key), and the str forms of one
            # dict's keys are unique, so the match is exact.  (The reference
            # also maps every int-looking segment to an int key, so
            # {1: a, "+1": b} came back as {1: b, "+1": b}.)
            by_key: Dict[str, Any] = {decode_key(k): v for k, v in vals.items()}
            for k in list(container.keys()):
                sk = str(k)
                if sk in by_key:
                    container[k] = by_key[sk]
                else:
                    del container[k]
        else:
            raise AssertionError(
                f"inflate() does not know how to inflate container of type "
                f"{type(container)} (path: {path}, container entry: {manifest.get(path)}).")
    return containers[root]
