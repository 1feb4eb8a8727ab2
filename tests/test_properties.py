"""Property tests (hypothesis) of the pure planning code every save and
restore depends on:

* the DTensor write plan (``io/sharded.py``: ``dim_index_runs`` ->
  ``runs_to_boxes`` -> ``split_for_replicas``) writes every global element
  exactly once, for any mix of ``Shard`` / ``_StridedShard`` / ``Replicate``
  placements on 1-3-D meshes;
* a restore into ANY other layout (``overlap_narrows`` of the saved boxes
  against the new local boxes) rebuilds every local tensor exactly, checked
  against a numpy model of the global tensor;
* the replicated-write partitioner (``plan_partition``) assigns every unit to
  one rank, is independent of dict order, and stays within one unit of the
  mean (the LPT bound);
* ``flatten`` / ``inflate`` round-trips nested containers with arbitrary
  str / int keys (``%``, ``/``, int-looking strings);
* the HSZ1 codec is lossless and the C++ coder matches the NumPy reference
  byte for byte on adversarial byte distributions (1 to 256 distinct high
  bytes, skewed weights, every element width).

The reference tests the same behaviour on hand-picked cases
(`/root/reference/tests/test_flatten.py`, `test_sharded_tensor_resharding.py`,
`test_partitioner.py`); these search the space.
"""

import os
from collections import OrderedDict
from itertools import product

import numpy as np
import pytest

hypothesis = pytest.importorskip("hypothesis")
from hypothesis import given, settings, strategies as st  # noqa: E402

from hipsnapshot.format.flatten import flatten, inflate  # noqa: E402
from hipsnapshot.io.sharded import (  # noqa: E402
    dim_index_runs,
    overlap_narrows,
    replica_index,
    runs_to_boxes,
    split_for_replicas,
)
from hipsnapshot.parallel.partitioner import plan_partition  # noqa: E402

SETTINGS = settings(max_examples=int(os.environ.get("HS_PROP_EXAMPLES", "150")), deadline=None)


# ---- DTensor layouts -------------------------------------------------------------


@st.composite
def layouts(draw, shape=None):
    """(global shape, mesh shape, placements)."""
    from torch.distributed.tensor.placement_types import Replicate, Shard, _StridedShard

    if shape is None:
        ndim = draw(st.integers(1, 3))
        shape = [draw(st.integers(0, 9)) for _ in range(ndim)]
    ndim = len(shape)
    mdims = draw(st.integers(1, 3))
    mesh = [draw(st.integers(1, 4)) for _ in range(mdims)]
    placements = []
    for _ in range(mdims):
        kind = draw(st.sampled_from(["shard", "replicate", "strided"]))
        d = draw(st.integers(0, ndim - 1))
        if kind == "shard":
            placements.append(Shard(d))
        elif kind == "replicate":
            placements.append(Replicate())
        else:
            placements.append(_StridedShard(d, split_factor=draw(st.integers(1, 4))))
    return shape, mesh, placements


def _coords(mesh):
    return product(*[range(n) for n in mesh])


def _local_index(runs):
    """Per dim, the global indices of the local tensor in local order."""
    return [np.concatenate([np.arange(g, g + ln) for g, ln in r]) if r else
            np.zeros(0, dtype=np.int64) for r in runs]


def _written_pieces(shape, mesh, placements, itemsize, min_split, glob):
    """Every (global offsets, sizes, data) box the ranks of this layout write."""
    pieces = []
    for coord in _coords(mesh):
        runs = dim_index_runs(shape, mesh, coord, placements)
        local = glob[np.ix_(*_local_index(runs))]
        j, r = replica_index(mesh, coord, placements)
        for lo, go, sz in split_for_replicas(runs_to_boxes(runs), j, r, itemsize, shape,
                                             min_split):
            if 0 in sz:
                continue
            sl = tuple(slice(o, o + s) for o, s in zip(lo, sz))
            pieces.append((go, sz, local[sl]))
    return pieces


@SETTINGS
@given(layouts(), st.sampled_from([1, 2, 4]), st.sampled_from([0, 8, 64, 1 << 30]))
def test_write_plan_writes_every_element_exactly_once(layout, itemsize, min_split):
    shape, mesh, placements = layout
    count = np.zeros(shape, dtype=np.int64)
    glob = np.arange(int(np.prod(shape)), dtype=np.int64).reshape(shape)
    for go, sz, data in _written_pieces(shape, mesh, placements, itemsize, min_split, glob):
        sl = tuple(slice(o, o + s) for o, s in zip(go, sz))
        count[sl] += 1
        # a box's bytes are the global tensor's bytes at its offsets
        assert np.array_equal(glob[sl], data)
    assert (count == 1).all(), (shape, mesh, placements, count)


@SETTINGS
@given(layouts(), st.sampled_from([1, 2, 4]))
def test_local_runs_match_local_shape_and_partition_each_dim(layout, itemsize):
    """The runs of each coordinate are disjoint, in range, and the Shard
    coordinates along a dim tile it (together with the replicas)."""
    shape, mesh, placements = layout
    for coord in _coords(mesh):
        runs = dim_index_runs(shape, mesh, coord, placements)
        for d, r in enumerate(runs):
            idx = _local_index([r])[0]
            assert len(set(idx.tolist())) == len(idx)
            assert ((idx >= 0) & (idx < shape[d])).all()
        boxes = runs_to_boxes(runs)
        assert sum(int(np.prod(sz)) for _l, _g, sz in boxes) == \
            int(np.prod([sum(ln for _g, ln in r) for r in runs]))


@SETTINGS
@given(st.data())
def test_restore_into_any_layout_rebuilds_every_local_tensor(data):
    """Save with one layout, restore into another (elastic resharding):
    every target local tensor is rebuilt exactly from the intersections the
    restore computes."""
    shape, mesh_a, pl_a = data.draw(layouts())
    _s, mesh_b, pl_b = data.draw(layouts(shape=shape))
    min_split = data.draw(st.sampled_from([0, 16, 1 << 30]))
    glob = np.arange(int(np.prod(shape)), dtype=np.int64).reshape(shape) + 1
    saved = _written_pieces(shape, mesh_a, pl_a, 8, min_split, glob)
    for coord in _coords(mesh_b):
        runs = dim_index_runs(shape, mesh_b, coord, pl_b)
        expect = glob[np.ix_(*_local_index(runs))]
        out = np.zeros_like(expect)
        cover = np.zeros(expect.shape, dtype=np.int64)
        for lo, go, sz in runs_to_boxes(runs):
            if 0 in sz:
                continue
            for sgo, ssz, sdata in saved:
                nar = overlap_narrows(sgo, ssz, go, sz)
                if nar is None:
                    continue
                src = tuple(slice(s, s + ln) for _d, s, _c, ln in nar)
                dst = tuple(slice(l0 + c, l0 + c + ln) for l0, (_d, _s, c, ln) in zip(lo, nar))
                out[dst] = sdata[src]
                cover[dst] += 1
        assert (cover == 1).all()
        assert np.array_equal(out, expect)


@given(st.lists(st.integers(0, 50), min_size=1, max_size=4),
       st.lists(st.integers(0, 50), min_size=1, max_size=4),
       st.lists(st.integers(0, 50), min_size=1, max_size=4),
       st.lists(st.integers(0, 50), min_size=1, max_size=4))
@SETTINGS
def test_overlap_narrows_is_the_box_intersection(so, ss, co, cs):
    n = min(len(so), len(ss), len(co), len(cs))
    so, ss, co, cs = so[:n], ss[:n], co[:n], cs[:n]
    nar = overlap_narrows(so, ss, co, cs)
    inter = [(max(a, c), min(a + b, c + d)) for a, b, c, d in zip(so, ss, co, cs)]
    if any(hi <= lo for lo, hi in inter):
        assert nar is None
        return
    assert nar is not None
    for (d, s_start, c_start, ln), (lo, hi) in zip(nar, inter):
        assert ln == hi - lo
        assert so[d] + s_start == lo and co[d] + c_start == lo


# ---- replicated-write partitioner ------------------------------------------------


@st.composite
def partition_inputs(draw):
    world = draw(st.integers(1, 8))
    rank_sizes = [draw(st.integers(0, 1000)) for _ in range(world)]
    npaths = draw(st.integers(0, 12))
    path_loads, subpart = {}, {}
    for i in range(npaths):
        key = f"p{draw(st.integers(0, 10 ** 6))}_{i}"
        path_loads[key] = [draw(st.integers(0, 500)) for _ in range(draw(st.integers(1, 5)))]
        subpart[key] = draw(st.booleans())
    return rank_sizes, path_loads, subpart


@SETTINGS
@given(partition_inputs())
def test_partition_assigns_every_unit_once_within_the_lpt_bound(inp):
    rank_sizes, path_loads, subpart = inp
    owner = plan_partition(rank_sizes, path_loads, subpart)
    expect_keys = {(p, i) for p, s in path_loads.items() for i in range(len(s))}
    assert set(owner) == expect_keys
    assert all(0 <= r < len(rank_sizes) for r in owner.values())
    # whole (non-subpartitionable) paths stay on one rank
    for p, s in path_loads.items():
        if not subpart[p]:
            assert len({owner[(p, i)] for i in range(len(s))}) == 1
    loads = list(rank_sizes)
    units = []
    for p, s in path_loads.items():
        if subpart[p]:
            units += s
        else:
            units.append(sum(s))
    for (p, i), r in owner.items():
        loads[r] += path_loads[p][i]
    # greedy LPT: the busiest rank ends within one unit of the mean (or is a
    # rank that started above it)
    mean = sum(loads) / len(loads)
    biggest = max(units, default=0)
    assert max(loads) <= max(max(rank_sizes), mean + biggest)
    # every rank computes the same plan, whatever order its dict is in
    shuffled = dict(reversed(list(path_loads.items())))
    assert plan_partition(rank_sizes, shuffled, subpart) == owner


# ---- flatten / inflate -----------------------------------------------------------

_keys = st.one_of(st.integers(-3, 12), st.text(alphabet="ab%/2+-0", min_size=0, max_size=4))
_leaves = st.one_of(st.integers(), st.text(max_size=3), st.none(), st.floats(allow_nan=False))


def _containers(children):
    def unique_str(d):
        return len({str(k) for k in d}) == len(d)

    return st.one_of(
        st.lists(children, max_size=4),
        st.dictionaries(_keys, children, max_size=4).filter(unique_str),
        st.dictionaries(_keys, children, max_size=4).filter(unique_str).map(
            lambda d: OrderedDict(d)),
    )


_trees = st.recursive(_leaves, _containers, max_leaves=20)


@SETTINGS
@given(st.dictionaries(st.text(alphabet="xyz/%", min_size=1, max_size=3), _trees, max_size=3),
       st.sampled_from(["0", "app", "a/b"]))
def test_flatten_inflate_round_trips_any_tree(tree, prefix):
    manifest, flat = flatten(tree, prefix)
    back = inflate(manifest, flat, prefix)
    assert back == tree
    assert type(back) is type(tree)


def test_inflate_int_key_next_to_an_int_looking_str_key():
    """The case the property test found: {1: a, "+1": b} used to come back
    with b under both keys (the reference has the same behaviour)."""
    tree = {1: "a", "+1": "b", "01": "c", -2: "d", "-02": "e"}
    manifest, flat = flatten(tree, "0")
    assert inflate(manifest, flat, "0") == tree


# ---- HSZ1 codec ------------------------------------------------------------------


@st.composite
def codec_inputs(draw):
    """Byte streams whose high bytes range from one value to all 256, with
    skewed weights: the dictionary, escape and Huffman paths all get hit."""
    w = draw(st.sampled_from([1, 2, 4, 8]))
    n = draw(st.integers(0, 12_000))
    alphabet = draw(st.integers(1, 256))
    seed = draw(st.integers(0, 2 ** 31 - 1))
    skew = draw(st.floats(0.0, 3.0))
    rng = np.random.default_rng(seed)
    p = (np.arange(1, alphabet + 1, dtype=np.float64)) ** -skew
    vals = rng.permutation(256)[:alphabet].astype(np.uint8)
    raw = rng.integers(0, 256, size=n, dtype=np.uint8)
    hi = vals[rng.choice(alphabet, size=n, p=p / p.sum())]
    if w > 1:
        raw[w - 1::w] = hi[w - 1::w]  # little endian: the high byte is the last
    else:
        raw[:] = hi
    frame = draw(st.sampled_from([512, 4096, 64 * 1024]))
    return raw.tobytes(), w, frame


@settings(max_examples=int(os.environ.get("HS_PROP_EXAMPLES", "60")), deadline=None)
@given(codec_inputs())
def test_hsz1_native_matches_reference_and_is_lossless(inp):
    from hipsnapshot.ops import codec

    raw, w, frame = inp
    ref = codec.encode_reference(raw, w, frame_bytes=frame)
    assert len(ref) <= codec.max_encoded_bytes(len(raw), frame)
    assert codec.decode_reference(ref) == raw
    nat = codec.encode_cpu(raw, w, frame, nthreads=3)
    assert nat.tobytes() == ref
    assert codec.decode_cpu(ref).tobytes() == raw
