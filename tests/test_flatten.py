"""flatten/inflate round trips (reference test strategy: tests/test_flatten.py)."""

from collections import OrderedDict

import pytest
import torch

from hipsnapshot.format.flatten import encode_key, flatten, inflate
from hipsnapshot.format.manifest import DictEntry, ListEntry, OrderedDictEntry


def _obj():
    return {
        "foo": 0,
        "bar": 1,
        "baz": [2, 3, {"qux": 4, "quxx": [5, OrderedDict(quuz=6, corge=[7, 8, 9])]}],
        "x/y": {"%a/b": 10},
        "": {"": []},
        "dict_with_colliding_keys": {"0": {"1": "foo", 1: "bar"}, 0: "baz"},
        "dict_with_mixed_type_keys": {0: {"0": "foo", 1: "bar"}, "1": "baz"},
        "long_list": list(range(100)),
    }


@pytest.mark.parametrize("prefix", ["", "prefix_without_slashes", "prefix/with/slashes"])
def test_flatten_inflate(prefix):
    obj = _obj()
    manifest, flattened = flatten(obj, prefix=prefix)
    p = encode_key(prefix)
    expected_manifest = {
        "baz": ListEntry(),
        "baz/2": DictEntry(keys=["qux", "quxx"]),
        "baz/2/quxx": ListEntry(),
        "baz/2/quxx/1": OrderedDictEntry(keys=["quuz", "corge"]),
        "baz/2/quxx/1/corge": ListEntry(),
        "x%2Fy": DictEntry(keys=["%a/b"]),
        "": DictEntry(keys=[""]),
        "/": ListEntry(),
        "dict_with_mixed_type_keys": DictEntry(keys=[0, "1"]),
        "dict_with_mixed_type_keys/0": DictEntry(keys=["0", 1]),
        "long_list": ListEntry(),
    }
    expected_manifest = {f"{p}/{k}": v for k, v in expected_manifest.items()}
    expected_manifest[p] = DictEntry(keys=list(obj.keys()))
    assert manifest == expected_manifest
    expected_flat = {
        "foo": 0, "bar": 1, "baz/0": 2, "baz/1": 3, "baz/2/qux": 4, "baz/2/quxx/0": 5,
        "baz/2/quxx/1/quuz": 6, "baz/2/quxx/1/corge/0": 7, "baz/2/quxx/1/corge/1": 8,
        "baz/2/quxx/1/corge/2": 9, "x%2Fy/%25a%2Fb": 10,
        "dict_with_colliding_keys": {"0": {"1": "foo", 1: "bar"}, 0: "baz"},
        "dict_with_mixed_type_keys/0/0": "foo", "dict_with_mixed_type_keys/0/1": "bar",
        "dict_with_mixed_type_keys/1": "baz",
    }
    expected_flat.update({f"long_list/{i}": i for i in range(100)})
    assert flattened == {f"{p}/{k}": v for k, v in expected_flat.items()}
    assert inflate(manifest, flattened, prefix=prefix) == obj


@pytest.mark.parametrize("prefix", ["", "p", "p/q"])
def test_non_flattenable_object(prefix):
    obj = {"0": 1, 0: 2}
    manifest, flattened = flatten(obj, prefix=prefix)
    assert manifest == {}
    assert flattened == {encode_key(prefix): obj}
    assert inflate(manifest, flattened, prefix=prefix) == obj


def test_leaf_and_tensors():
    t = torch.arange(4)
    manifest, flattened = flatten(t, prefix="x")
    assert manifest == {} and flattened["x"] is t
    m, f = flatten({"a": [t, {"b": t}]}, prefix="s")
    out = inflate(m, f, prefix="s")
    assert out["a"][0] is t and out["a"][1]["b"] is t


def test_inflate_drops_missing_children():
    m, f = flatten({"a": 1, "b": 2}, prefix="s")
    del f["s/b"]
    assert inflate(m, f, prefix="s") == {"a": 1}


def test_deep_nesting_no_recursion_limit():
    obj = cur = {}
    for _ in range(3000):
        cur["n"] = {}
        cur = cur["n"]
    cur["leaf"] = 1
    m, f = flatten(obj, prefix="d")
    assert len(f) == 1
    out = inflate(m, f, prefix="d")
    for _ in range(3000):
        out = out["n"]
    assert out == {"leaf": 1}


def test_inflate_other_prefix_ignored():
    m1, f1 = flatten({"a": 1}, prefix="x")
    m2, f2 = flatten({"a": 2}, prefix="xy")
    assert inflate({**m1, **m2}, {**f1, **f2}, prefix="x") == {"a": 1}
