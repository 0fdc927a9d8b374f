"""Struct (OPTIONAL group) validity and shared ancestor arrays (the struct half).

Column.getNextData (schema.go:216-260) assembles a group from its children: the group is nil
unless some child is non-nil or is defined exactly one level below its own maximum, i.e. unless
the leaf's definition level reaches the group's own level. Column.getData (:283-312) wraps
REPEATED groups into lists, and ColumnStore.get (data_store.go:262-309) makes a leaf null iff
dLevel < maxD. In columnar form a group g at list depth j (REPEATED nodes above it) has one entry
per element of list depth j (per record at depth 0) and is non-null iff def >= its own level.

`tree_ref` restates that function from the leaf's levels and the repetition types of the nodes
on its path as the ORACLE's schema walk reports them (oracle.c read_group_schema /
read_column_schema, schema.go:893-990) — not from the product's schema walk. It is pinned against
pyarrow's StructArray / ListArray / MapArray validity on the struct fixtures (an independent
Dremel -> Arrow implementation) and against the reference test document's Links group, written
out by hand below. The GPU (k_nest_emit, k_group_flat) must equal `tree_ref` on the oracle's levels.
"""
import io

import numpy as np
import pytest

import pqgpu

import pqtest
import py_oracle as O
import test_ref_goldens as G
from pqtest import schema_levels
from test_nested import nested_ref

STRUCT_FIXTURES = ["struct_v1", "struct_v2"]


def tree_ref(rep, dfn, node_reps):
    """(list levels [(offsets, validity)], element validity, groups [(node, validity)])."""
    lists, groups, max_def = schema_levels(node_reps)
    rep = np.zeros(len(dfn), np.int64) if rep is None or not len(lists) else np.asarray(rep, np.int64)
    dfn = np.asarray(dfn, np.int64)
    if lists:
        levels, elem = nested_ref(rep, dfn, max_def, [x[0] for x in lists], [x[1] for x in lists])
    else:
        levels, elem = [], (dfn == max_def).astype(np.uint8)
    D = [0] + [x[1] for x in lists]
    out = []
    for dg, j, node in groups:
        ent = (rep <= j) & (dfn >= D[j])  # an element of list depth j (a record at 0) starts here
        out.append((node, (dfn[ent] >= dg).astype(np.uint8)))
    return levels, elem, out


def _oracle_chunks(data):
    of = O.File(data)
    for rg in range(of.num_row_groups):
        for col in range(of.num_columns):
            ci = of.column_info(col)
            yield rg, col, ci.path.decode(), list(ci.node_rep[:ci.path_len]), of.read_chunk(rg, col)


# ---------------------------------------------------------------------------------------------
# CPU: the restatement against pyarrow, the product's schema walk against the oracle's
# ---------------------------------------------------------------------------------------------
def _arrow_group_validity(tbl, path):
    """pyarrow's validity of the Parquet group at dotted `path` of the struct fixtures, over the
    entries of its list depth (pyarrow propagates a parent's nulls into its children)."""
    parts = path.split(".")
    arr = tbl.column(parts[0]).combine_chunks()
    if len(parts) == 1:
        return np.asarray(arr.is_valid(), np.uint8)
    if parts[0] == "s" and parts[1] == "l":  # LIST-annotated group inside struct s
        return np.asarray(arr.field("l").is_valid(), np.uint8)
    if parts[0] == "t" and parts[1] == "u":
        return np.asarray(arr.field("u").is_valid(), np.uint8)
    if parts[0] == "ls" and parts[1:] == ["list", "element"]:  # struct elements of list ls
        o = np.asarray(arr.offsets)
        return np.asarray(arr.values.slice(o[0], o[-1] - o[0]).is_valid(), np.uint8)
    raise KeyError(path)


@pytest.mark.parametrize("name", STRUCT_FIXTURES)
def test_tree_ref_matches_pyarrow(name):
    import pyarrow.parquet as pq
    data = pqtest.load(name)
    pf = pq.ParquetFile(io.BytesIO(data))
    seen = set()
    for rg, col, path, reps, r in _oracle_chunks(data):
        tbl = pf.read_row_group(rg)
        _levels, elem, groups = tree_ref(r.rep_levels, r.def_levels, reps)
        parts = path.split(".")
        for node, v in groups:
            gpath = ".".join(parts[: node + 1])
            np.testing.assert_array_equal(v, _arrow_group_validity(tbl, gpath), err_msg=f"{name} rg{rg} {path} group {gpath}")
            seen.add(gpath)
    assert seen == {"s", "s.l", "ls", "ls.list.element", "t", "t.u", "mm"}, seen


def test_tree_ref_links_group():
    """The reference's Dremel document (data_store_test.go:227-345): Links is present in both
    records (r1: Forward only; r2: Backward and Forward)."""
    data = G.build("dremel")
    for _rg, _col, path, reps, r in _oracle_chunks(data):
        if not path.startswith("Links."):
            continue
        _levels, _elem, groups = tree_ref(r.rep_levels, r.def_levels, reps)
        assert [(n, list(v)) for n, v in groups] == [(0, [1, 1])], path


@pytest.mark.parametrize("name", STRUCT_FIXTURES + ["cfg4_small"])
def test_schema_groups_match_oracle(name):
    """pqgpu_file_column's list and group thresholds equal those derived from the oracle's walk."""
    import pqgpu
    data = pqtest.load(name)
    f = pqgpu.File(data)
    of = O.File(data)
    for col in range(f.num_columns):
        ci, oi = f.column(col), of.column_info(col)
        lists, groups, max_def = schema_levels(list(oi.node_rep[:oi.path_len]))
        assert (ci.max_def, ci.max_rep) == (max_def, len(lists))
        assert [(ci.list_null_def[k], ci.list_def[k], ci.list_node[k]) for k in range(ci.max_rep)] == lists
        assert [(ci.group_def[g], ci.group_depth[g], ci.group_node[g]) for g in range(ci.num_groups)] == groups


# ---------------------------------------------------------------------------------------------
# GPU
# ---------------------------------------------------------------------------------------------
def _decode_all(gpu_ctx, data):
    import pqgpu
    f = pqgpu.File(data)
    b = pqgpu.Batch(gpu_ctx)
    ids = {}
    for rg in range(f.num_row_groups):
        for col in range(f.num_columns):
            cid, e = b.add_file_chunk(f, rg, col)
            assert e is None, e
            ids[(rg, col)] = cid
    b.decode()
    assert b.sync() is None
    return f, b, ids


@pytest.mark.gpu
@pytest.mark.parametrize("name", STRUCT_FIXTURES + ["cfg4_small", "cfg4_v2", "types_v1", "edge_nulls_v2"])
def test_gpu_groups_vs_tree_ref(gpu_ctx, nest_mode, name):
    data = pqtest.load(name)
    f, b, ids = _decode_all(gpu_ctx, data)
    for rg, col, path, reps, o in _oracle_chunks(data):
        r = b.result(ids[(rg, col)])
        levels, elem, groups = tree_ref(o.rep_levels, o.def_levels, reps)
        where = f"{name} rg{rg} {path}"
        parts = path.split(".")
        assert [p for p, _ in r.groups] == [".".join(parts[: n + 1]) for n, _ in groups], where
        for (gp, gv), (_n, want) in zip(r.groups, groups):
            np.testing.assert_array_equal(gv, want, err_msg=f"{where} group {gp}")
        if levels:
            assert len(r.nested) == len(levels), where
            for k, ((go, gvl), (wo, wv)) in enumerate(zip(r.nested, levels)):
                np.testing.assert_array_equal(np.asarray(go, np.int64), wo, err_msg=f"{where} L{k} offsets")
                np.testing.assert_array_equal(gvl, wv, err_msg=f"{where} L{k} validity")
            np.testing.assert_array_equal(r.element_validity, elem, err_msg=f"{where} elements")
    b.close()


@pytest.mark.gpu
@pytest.mark.parametrize("v2", [False, True])
def test_gpu_links_group(gpu_ctx, nest_mode, v2):
    data = G.build("dremel", v2)
    f, b, ids = _decode_all(gpu_ctx, data)
    paths = f.column_paths()
    for (rg, col), cid in ids.items():
        if paths[col].startswith("Links."):
            r = b.result(cid)
            assert [(p, list(v)) for p, v in r.groups] == [("Links", [1, 1])], paths[col]
    b.close()


def _sibling_pairs(paths):
    return [(a, c) for a in range(len(paths)) for c in range(a + 1, len(paths))
            if paths[a].split(".")[0] == paths[c].split(".")[0]]


@pytest.mark.gpu
@pytest.mark.parametrize("name", STRUCT_FIXTURES + ["cfg4_small"])
def test_gpu_share_ancestors(gpu_ctx, nest_mode, name):
    """Sibling leaves of one group (a MAP's key and value; struct fields) decode identical arrays
    for their common ancestors; after the check the second leaf's result carries the first's
    (one offsets array per shared list level, one bitmap per shared group)."""
    import ctypes
    data = pqtest.load(name)
    f, b, ids = _decode_all(gpu_ctx, data)
    paths = f.column_paths()
    pairs = _sibling_pairs(paths)
    assert pairs
    for rg in range(f.num_row_groups):
        for a, c in pairs:
            ca, cc = ids[(rg, a)], ids[(rg, c)]
            before = b.result(cc)
            assert b.share_ancestors(ca, cc), (paths[a], paths[c])
            ra, rc = b.result(ca, copy=False), b.result(cc, copy=False)
            common = 0
            for x, y in zip(paths[a].split(".")[:-1], paths[c].split(".")[:-1]):
                if x != y:
                    break
                common += 1
            ci = f.column(a)
            nl = sum(1 for k in range(ci.max_rep) if ci.list_node[k] < common)
            ng = sum(1 for g in range(ci.num_groups) if ci.group_node[g] < common)
            for k in range(nl):
                assert ctypes.cast(ra.lvl_offsets[k], ctypes.c_void_p).value == \
                    ctypes.cast(rc.lvl_offsets[k], ctypes.c_void_p).value, (paths[c], k)
            for g in range(ng):
                assert ra.group_validity[g] == rc.group_validity[g], (paths[c], g)
            after = b.result(cc)  # same contents through the shared arrays
            for (o1, v1), (o2, v2) in zip(before.nested, after.nested):
                np.testing.assert_array_equal(o1, o2)
                np.testing.assert_array_equal(v1, v2)
            for (p1, g1), (p2, g2) in zip(before.groups, after.groups):
                assert p1 == p2
                np.testing.assert_array_equal(g1, g2)
    b.close()


@pytest.mark.gpu
def test_gpu_share_ancestors_detects_mismatch(gpu_ctx):
    """A MAP whose key and value leaves disagree about the entries (a corrupt or inconsistent file):
    the check reports it and shares nothing."""
    data = G.build("map_mismatch")
    f, b, ids = _decode_all(gpu_ctx, data)
    paths = f.column_paths()
    ka, va = paths.index("m.key_value.key"), paths.index("m.key_value.value")
    assert not b.share_ancestors(ids[(0, ka)], ids[(0, va)])
    r = b.result(ids[(0, va)], copy=False)
    rk = b.result(ids[(0, ka)], copy=False)
    assert r.lvl_offsets[0] != rk.lvl_offsets[0]
    b.close()


def _three_leaf_file():
    """a: list<struct<x: int32, b: list<struct<y: int32, z: int32>>>> with nulls at every level:
    leaf x has one list level, leaves b.y and b.z two, and all three share a's list."""
    import pyarrow as pa
    import pyarrow.parquet as pq
    rng = np.random.default_rng(77)
    rows = []
    for _ in range(3000):
        if rng.random() < 0.05:
            rows.append(None)
            continue
        elems = []
        for _ in range(int(rng.integers(0, 4))):
            if rng.random() < 0.1:
                elems.append(None)
                continue
            bl = None if rng.random() < 0.1 else [
                None if rng.random() < 0.1 else {"y": None if rng.random() < 0.2 else int(rng.integers(0, 1000)),
                                                  "z": int(rng.integers(0, 1000))}
                for _ in range(int(rng.integers(0, 4)))]
            elems.append({"x": None if rng.random() < 0.2 else int(rng.integers(0, 1000)), "b": bl})
        rows.append(elems)
    inner = pa.struct([("y", pa.int32()), ("z", pa.int32())])
    typ = pa.list_(pa.struct([("x", pa.int32()), ("b", pa.list_(inner))]))
    buf = io.BytesIO()
    pq.write_table(pa.table({"a": pa.array(rows, typ)}), buf, row_group_size=1000, data_page_size=2048,
                   use_dictionary=False)
    return buf.getvalue()


@pytest.mark.gpu
def test_gpu_share_ancestors_mixed_depths(gpu_ctx, nest_mode):
    """Leaf b.y first shares one list level with the shallower leaf x, then two list levels with its
    sibling b.z: b.z must take levels it shares with b.y from b.y (whose own result resolves level 0
    through x), not from the chain's root x, which has no level 1. Every result keeps its contents."""
    data = _three_leaf_file()
    f, b, ids = _decode_all(gpu_ctx, data)
    paths = f.column_paths()
    ix, iy, iz = (paths.index(p) for p in ("a.list.element.x", "a.list.element.b.list.element.y",
                                           "a.list.element.b.list.element.z"))
    for rg in range(f.num_row_groups):
        cx, cy, cz = ids[(rg, ix)], ids[(rg, iy)], ids[(rg, iz)]
        before = {c: b.result(c) for c in (cx, cy, cz)}
        assert b.share_ancestors(cx, cy)
        assert b.share_ancestors(cy, cz)
        assert b.share_ancestors(cz, cx)  # cz already follows cx through cy: no link back
        for c in (cx, cy, cz):
            r0, r1 = before[c], b.result(c)
            assert len(r0.nested) == len(r1.nested)
            for (o1, v1), (o2, v2) in zip(r0.nested, r1.nested):
                np.testing.assert_array_equal(o1, o2)
                np.testing.assert_array_equal(v1, v2)
            assert [p for p, _ in r0.groups] == [p for p, _ in r1.groups]
            for (_p1, g1), (_p2, g2) in zip(r0.groups, r1.groups):
                np.testing.assert_array_equal(g1, g2)
    b.close()


@pytest.mark.gpu
def test_gpu_share_ancestors_no_cycles(gpu_ctx):
    """Sharing links stay acyclic: a leaf cannot share with itself (an argument error), sharing a
    pair in both directions leaves every result readable with the same
    contents (chunk_result follows share_from to a root; host.cpp links to the root)."""
    data = pqtest.load("cfg4_small")
    f, b, ids = _decode_all(gpu_ctx, data)
    paths = f.column_paths()
    ka, va = ids[(0, paths.index("m.key_value.key"))], ids[(0, paths.index("m.key_value.value"))]
    with pytest.raises(pqgpu.DecodeError):
        b.share_ancestors(ka, ka)
    before_k, before_v = b.result(ka), b.result(va)
    assert b.share_ancestors(ka, va)
    assert b.share_ancestors(va, ka)  # already shared the other way: no link back
    for r0, r1 in ((before_k, b.result(ka)), (before_v, b.result(va))):
        for (o1, v1), (o2, v2) in zip(r0.nested, r1.nested):
            np.testing.assert_array_equal(o1, o2)
            np.testing.assert_array_equal(v1, v2)
    b.close()
