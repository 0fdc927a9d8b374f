"""Arrow-style nested arrays of repeated leaves (nested.hip): per REPEATED node on the leaf's path,
list offsets into the next level (innermost: into the leaf's element slots) and list validity (a
null list and an empty list both have no children), plus element validity.

The arrays are a function of the leaf's (rep, def) levels and its path (the levels themselves are
pinned against the reference's tests and the oracle elsewhere). `nested_ref` restates that
function slot by slot (the record assembly rules of ColumnStore.get data_store.go:262-309 and
Column.getData schema.go:216-312: rLevel < maxR starts a new object, dLevel < maxD is a null or
absent value), and is pinned here by (1) the Dremel / Twitter documents of the reference's tests
(data_store_test.go:227-390), whose nesting is written out by hand below, and (2) pyarrow's own
ListArray / MapArray reading of the cfg4 fixtures (an independent Dremel -> Arrow implementation).
The thresholds come from the oracle's schema walk (pqtest.schema_levels over the path's repetition
types), independent of the product's. The GPU must equal `nested_ref` applied to the oracle's levels."""
import io

import numpy as np
import pytest

import pqtest
import py_oracle as O
import test_ref_goldens as G


def nested_ref(rep, dfn, max_def, list_null_def, list_def):
    """[(offsets, validity) per list level, outermost first], element validity."""
    R = len(list_def)
    offs = [[] for _ in range(R)]
    valid = [[] for _ in range(R)]
    cnt = [0] * (R + 1)  # lists per level 1..R, then leaf elements
    elem = []
    for r, d in zip(rep, dfn):
        for k in range(1, R + 1):
            if r < k and d >= (list_def[k - 2] if k >= 2 else 0):
                offs[k - 1].append(cnt[k])  # children of the level-k list before this slot
                valid[k - 1].append(int(d >= list_null_def[k - 1]))
                cnt[k - 1] += 1
        if d >= list_def[R - 1]:
            elem.append(int(d == max_def))
            cnt[R] += 1
    for k in range(R):
        offs[k].append(cnt[k + 1])
    return [(np.array(o, np.int64), np.array(v, np.uint8)) for o, v in zip(offs, valid)], np.array(elem, np.uint8)


# Hand-derived nesting of the reference's documents: path -> (levels [(offsets, validity)], element validity)
GOLDEN = {
    ("dremel", "Links.Backward"): ([([0, 0, 2], [1, 1])], [1, 1]),  # r1: Links present, no Backward (empty)
    ("dremel", "Links.Forward"): ([([0, 3, 4], [1, 1])], [1, 1, 1, 1]),
    ("dremel", "Name.Language.Code"): ([([0, 3, 4], [1, 1]), ([0, 2, 2, 3, 3], [1, 1, 1, 1])], [1, 1, 1]),
    ("dremel", "Name.Language.Country"): ([([0, 3, 4], [1, 1]), ([0, 2, 2, 3, 3], [1, 1, 1, 1])], [1, 0, 1]),
    ("dremel", "Name.URL"): ([([0, 3, 4], [1, 1])], [1, 1, 0, 1]),
    ("twitter", "level1.level2"): ([([0, 2, 4], [1, 1]), ([0, 3, 7, 8, 10], [1, 1, 1, 1])], [1] * 10),
    ("one_repeated", "DocID"): ([([0, 2, 2], [1, 1])], [1, 1]),
}


def _levels_of(data, col):
    """The list thresholds from the ORACLE's schema walk (the repetition type of every node on the
    leaf's path, oracle.c read_group_schema), not from the product's: (null defs, defs, maxD)."""
    oi = O.File(data).column_info(col)
    lists, _groups, max_def = pqtest.schema_levels(list(oi.node_rep[:oi.path_len]))
    return [x[0] for x in lists], [x[1] for x in lists], max_def


def _check_nested(got_levels, got_elem, want_levels, want_elem, where):
    assert len(got_levels) == len(want_levels), where
    for k, ((go, gv), (wo, wv)) in enumerate(zip(got_levels, want_levels)):
        np.testing.assert_array_equal(np.asarray(go, np.int64), np.asarray(wo, np.int64), err_msg=f"{where} L{k} offsets")
        np.testing.assert_array_equal(np.asarray(gv, np.uint8), np.asarray(wv, np.uint8), err_msg=f"{where} L{k} validity")
    np.testing.assert_array_equal(np.asarray(got_elem, np.uint8), np.asarray(want_elem, np.uint8), err_msg=f"{where} elements")


@pytest.mark.parametrize("doc,path", sorted(GOLDEN))
def test_ref_documents(doc, path):
    """nested_ref on the reference tests' levels gives the documents' nesting."""
    import pqgpu
    data = G.build(doc)
    f = pqgpu.File(data)
    col = f.column_paths().index(path)
    lnd, ld, md = _levels_of(data, col)
    _, cols, _ = G.DOCS[doc]
    _, _, _, _, dl, rl = cols[col]
    got_levels, got_elem = nested_ref(rl, dl, md, lnd, ld)
    want_levels, want_elem = GOLDEN[(doc, path)]
    _check_nested(got_levels, got_elem, want_levels, want_elem, f"{doc} {path}")


def _nested_fixtures():
    return [n for n in pqtest.ALL if n.startswith("cfg4")]


@pytest.mark.parametrize("name", _nested_fixtures())
def test_ref_matches_pyarrow(name):
    """nested_ref on the oracle's levels equals pyarrow's list / map offsets and validity."""
    import pyarrow.parquet as pq
    import pqgpu
    data = pqtest.load(name)
    f = pqgpu.File(data)
    of = O.File(data)
    pf = pq.ParquetFile(io.BytesIO(data))
    paths = f.column_paths()
    for rg in range(f.num_row_groups):
        tbl = pf.read_row_group(rg)
        for col, path in enumerate(paths):
            ci = f.column(col)
            if ci.max_rep == 0:
                continue
            r = of.read_chunk(rg, col)
            lnd, ld, md = _levels_of(data, col)
            levels, elem = nested_ref(r.rep_levels, r.def_levels, md, lnd, ld)
            arr = tbl.column(path.split(".")[0]).combine_chunks()
            offs = np.asarray(arr.offsets, np.int64)
            np.testing.assert_array_equal(levels[0][0], offs - offs[0], err_msg=f"{name} rg{rg} {path} offsets")
            np.testing.assert_array_equal(levels[0][1], np.asarray(arr.is_valid(), np.uint8),
                                          err_msg=f"{name} rg{rg} {path} validity")
            child = arr.values if not hasattr(arr, "keys") else (arr.keys if path.endswith(".key") else arr.items)
            child = child.slice(offs[0], offs[-1] - offs[0])
            np.testing.assert_array_equal(elem, np.asarray(child.is_valid(), np.uint8),
                                          err_msg=f"{name} rg{rg} {path} elements")


def _gpu_nested_all(gpu_ctx, data):
    import pqgpu
    f = pqgpu.File(data)
    b = pqgpu.Batch(gpu_ctx)
    ids = {}
    for rg in range(f.num_row_groups):
        for col in range(f.num_columns):
            ids[(rg, col)] = b.add_file_chunk(f, rg, col)[0]
    b.decode()
    b.sync()
    return f, b, ids


@pytest.mark.gpu
@pytest.mark.parametrize("doc", sorted({d for d, _ in GOLDEN}))
@pytest.mark.parametrize("v2", [False, True])
def test_gpu_ref_documents(gpu_ctx, nest_mode, doc, v2):
    f, b, ids = _gpu_nested_all(gpu_ctx, G.build(doc, v2))
    for (rg, col), cid in ids.items():
        path = f.column_paths()[col]
        if (doc, path) not in GOLDEN:
            continue
        r = b.result(cid)
        want_levels, want_elem = GOLDEN[(doc, path)]
        _check_nested(r.nested, r.element_validity, want_levels, want_elem, f"gpu {doc} {path}")
    b.close()


@pytest.mark.gpu
@pytest.mark.parametrize("name", _nested_fixtures() + ["edge_nulls_v1", "types_v2"])
def test_gpu_nested_vs_ref(gpu_ctx, nest_mode, name):
    if name not in pqtest.ALL:
        pytest.skip("fixture absent")
    data = pqtest.load(name)
    of = O.File(data)
    f, b, ids = _gpu_nested_all(gpu_ctx, data)
    for (rg, col), cid in ids.items():
        ci = f.column(col)
        r = b.result(cid)
        if ci.max_rep == 0:
            assert not r.nested
            continue
        o = of.read_chunk(rg, col)
        lnd, ld, md = _levels_of(data, col)
        want_levels, want_elem = nested_ref(o.rep_levels, o.def_levels, md, lnd, ld)
        _check_nested(r.nested, r.element_validity, want_levels, want_elem, f"{name} rg{rg} col{col}")
    b.close()


def _deep_file(version):
    """struct<ll: list<list<int32>>> with nulls at every level (maxR 2, maxD 6: the levels take more
    than a nibble per slot, so k_nest_count packs them as bytes), small pages so that pages share
    fill tiles, V1 or V2 pages."""
    import pyarrow as pa
    import pyarrow.parquet as pq
    rng = np.random.default_rng(11)
    recs = []
    for _ in range(40_000):
        if rng.random() < 0.05:
            recs.append(None)
            continue
        if rng.random() < 0.05:
            recs.append({"ll": None})
            continue
        outer = []
        for _ in range(int(rng.integers(0, 5))):
            if rng.random() < 0.08:
                outer.append(None)
                continue
            outer.append([None if rng.random() < 0.1 else int(rng.integers(-1000, 1000))
                          for _ in range(int(rng.integers(0, 6)))])
        recs.append({"ll": outer})
    t = pa.table({"s": pa.array(recs, type=pa.struct([("ll", pa.list_(pa.list_(pa.int32())))]))})
    buf = io.BytesIO()
    # (uncompressed: pyarrow's V2 pages whose values do not shrink are stored with is_compressed
    # false, which the reference still hands to the codec: SURVEY App. A Q5, both readers fail it)
    pq.write_table(t, buf, use_dictionary=False, data_page_size=6000, data_page_version=version,
                   row_group_size=25_000, write_statistics=False, compression="NONE")
    return buf.getvalue()


@pytest.mark.gpu
@pytest.mark.parametrize("version", ["1.0", "2.0"])
def test_gpu_deep_nesting(gpu_ctx, nest_mode, version):
    """Nested arrays, levels and values of a two-list-level leaf with maxD 6 (byte-packed levels in
    k_nest_count / k_nest_emit) against the oracle, over pages that share fill tiles."""
    data = _deep_file(version)
    of = O.File(data)
    f, b, ids = _gpu_nested_all(gpu_ctx, data)
    for (rg, col), cid in ids.items():
        r = b.result(cid)
        o = of.read_chunk(rg, col)
        assert not isinstance(o, O.OracleError), o
        pqtest.assert_chunk_equal(r, o, f"deep {version} rg{rg} col{col}")
        lnd, ld, md = _levels_of(data, col)
        assert len(ld) == 2 and md == 6, (ld, md)
        want_levels, want_elem = nested_ref(o.rep_levels, o.def_levels, md, lnd, ld)
        _check_nested(r.nested, r.element_validity, want_levels, want_elem, f"deep {version} rg{rg} col{col}")
    b.close()


def test_deep_file_levels():
    """The deep-nesting fixture has the intended shape (CPU: the oracle's levels and schema walk)."""
    data = _deep_file("1.0")
    of = O.File(data)
    r = of.read_chunk(0, 0)
    assert not isinstance(r, O.OracleError), r
    lnd, ld, md = _levels_of(data, 0)
    assert md == 6 and len(ld) == 2
    assert int(np.max(r.def_levels)) == 6 and int(np.max(r.rep_levels)) == 2
    assert len(r.def_levels) > 8192 * 4  # several fill tiles per chunk


def _b2b_file(bad_page=None):
    """LIST<INT32> (optional list, optional elements: maxR 1, maxD 3) and a MAP-style dictionary
    BYTE_ARRAY key leaf (maxR 1, maxD 2), written as V1 pages without statistics, so the batch takes
    the serial schedule (cfg4's); the level streams are single bit-packed runs.
    bad_page: that data page of the list leaf gets a definition stream starting with an empty RLE run
    (hybrid_decoder.go:159-161)."""
    import os
    import struct
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(pqtest.GOLDEN), "..", "tools"))
    import rawpq
    rng = np.random.default_rng(23)
    vocab = sorted({bytes(rng.integers(97, 123, int(rng.integers(1, 24)), dtype=np.uint8)) for _ in range(300)})
    n_rec, per_page = 12_000, 1_500
    lpages, kpages, lslots, kslots = [], [rawpq.dict_page_ref("BYTE_ARRAY", vocab)], 0, 0
    for p0 in range(0, n_rec, per_page):
        lr, ld, lv, kr, kd, ki = [], [], [], [], [], []
        for _ in range(per_page):
            u = rng.random()
            if u < 0.08:
                lr.append(0), ld.append(0)
            elif u < 0.15:
                lr.append(0), ld.append(1)
            else:
                for j in range(int(rng.integers(1, 7))):
                    lr.append(0 if j == 0 else 1)
                    if rng.random() < 0.1:
                        ld.append(2)
                    else:
                        ld.append(3)
                        lv.append(int(rng.integers(-(1 << 31), 1 << 31)))
            u = rng.random()
            if u < 0.05:
                kr.append(0), kd.append(0)
            elif u < 0.1:
                kr.append(0), kd.append(1)
            else:
                for j in range(int(rng.integers(1, 5))):
                    kr.append(0 if j == 0 else 1), kd.append(2), ki.append(int(rng.integers(0, len(vocab))))
        page = len(lpages)
        if page == bad_page:  # rep stream as usual, the def stream: varint 0 (an empty RLE run), value byte
            body = rawpq.levels_v1_ref(lr, 1) + struct.pack("<I", 2) + b"\x00\x03" + rawpq.plain_encode("INT32", lv)
            dph = [(1, rawpq.I32, len(lr)), (2, rawpq.I32, rawpq.ENC["PLAIN"]), (3, rawpq.I32, rawpq.ENC["RLE"]),
                   (4, rawpq.I32, rawpq.ENC["RLE"])]
            lpages.append(rawpq._page(0, body, 5, dph))
        else:
            lpages.append(rawpq.data_page_v1_ref(len(lr), "PLAIN", rawpq.plain_encode("INT32", lv), def_levels=ld,
                                                 max_def=3, rep_levels=lr, max_rep=1))
        kpages.append(rawpq.data_page_v1_ref(len(kr), "RLE_DICTIONARY", rawpq.dict_values_section(ki, len(vocab)),
                                             def_levels=kd, max_def=2, rep_levels=kr, max_rep=1))
        lslots += len(lr)
        kslots += len(kr)
    schema = [[(4, rawpq.BIN, "schema"), (5, rawpq.I32, 2)],
              rawpq.schema_group("l", "OPTIONAL", 1), rawpq.schema_group("list", "REPEATED", 1),
              rawpq.schema_leaf("element", "INT32", "OPTIONAL"),
              rawpq.schema_group("m", "OPTIONAL", 1), rawpq.schema_group("key_value", "REPEATED", 1),
              rawpq.schema_leaf("key", "BYTE_ARRAY", "REQUIRED")]
    return rawpq.write_file_schema(schema, [("l.list.element", "INT32"), ("m.key_value.key", "BYTE_ARRAY")],
                                   [(n_rec, [(lpages, lslots, False), (kpages, kslots, True)])])


def test_b2b_file_shape():
    """The back-to-back fixtures decode in the oracle as intended: the good file whole, the bad one
    with the reference's empty-RLE-run error on the list leaf's page 2 and the map leaf intact."""
    good = pqtest.oracle_decode(_b2b_file())
    assert all(not isinstance(r, O.OracleError) for _, _, r in good)
    assert all(int(np.max(r.rep_levels)) == 1 for _, _, r in good)
    bad = pqtest.oracle_decode(_b2b_file(bad_page=2))
    assert isinstance(bad[0][2], O.OracleError) and bad[0][2].code == 3 and bad[0][2].page == 2
    assert not isinstance(bad[1][2], O.OracleError)


@pytest.mark.gpu
@pytest.mark.parametrize("bad_page", [None, 2])
def test_gpu_back_to_back_decodes(gpu_ctx, nest_mode, bad_page):
    """Three decodes queued back to back, then one sync (the benchmark's pattern), then decode + sync
    pairs: every chunk equals the oracle (levels, values, nested arrays) after each, and a level
    error is reported with the reference's code and page every time."""
    import pqgpu
    data = _b2b_file(bad_page)
    orc = pqtest.oracle_decode(data)
    f = pqgpu.File(data)
    b = pqgpu.Batch(gpu_ctx)
    ids = [b.add_file_chunk(f, 0, c)[0] for c in range(2)]
    for rounds in (3, 1, 1):
        for _ in range(rounds):
            b.decode()
        e = b.sync()
        for (rg, col, o), cid in zip(orc, ids):
            if isinstance(o, O.OracleError):
                assert e is not None and (e.code, e.page) == (o.code, o.page), (e, o)
                continue
            r = b.result(cid)
            pqtest.assert_chunk_equal(r, o, f"back-to-back col{col}")
            lnd, ld, md = _levels_of(data, col)
            want_levels, want_elem = nested_ref(o.rep_levels, o.def_levels, md, lnd, ld)
            _check_nested(r.nested, r.element_validity, want_levels, want_elem, f"back-to-back col{col}")
        if bad_page is None:
            assert e is None, e
    b.close()


@pytest.mark.gpu
def test_gpu_batch_reuse_bitmaps(gpu_ctx, nest_mode):
    """The validity bitmaps OR-written at shared edge words are zeroed by the first decode after an
    upload only (host.cpp bm_zeroed). One batch reused for different files (pqgpu_batch_reset, then
    new chunks and a new upload) must zero them again: every file's nested arrays and validity equal
    the oracle's on each of two decodes, whatever the previous file left in the arena."""
    import pqgpu
    b = pqgpu.Batch(gpu_ctx)
    for data in (_b2b_file(None), pqtest.load("cfg4_small"), _b2b_file(2), _b2b_file(None)):
        orc = pqtest.oracle_decode(data)
        f = pqgpu.File(data)
        ids = {(rg, col): b.add_file_chunk(f, rg, col)[0] for rg in range(f.num_row_groups) for col in range(f.num_columns)}
        for _ in range(2):
            b.decode()
            e = b.sync()
            for rg, col, o in orc:
                if isinstance(o, O.OracleError):
                    assert e is not None
                    g = b.status(ids[(rg, col)])
                    assert g is not None and (g.code, g.page) == (o.code, o.page), (g, o)
                    continue
                r = b.result(ids[(rg, col)])
                pqtest.assert_chunk_equal(r, o, f"reuse rg{rg} col{col}")
                if r.nested:
                    lnd, ld, md = _levels_of(data, col)
                    want_levels, want_elem = nested_ref(o.rep_levels, o.def_levels, md, lnd, ld)
                    _check_nested(r.nested, r.element_validity, want_levels, want_elem, f"reuse rg{rg} col{col}")
        b.reset()
    b.close()


TORN_SCRIPT = r"""
import sys
sys.path[:0] = sys.argv[1:4]
import numpy as np
import pqgpu, pqtest, py_oracle as O
import test_nested as T
ctx = pqgpu.Context(0)
torn = over = 0
for name, data in (("cfg4_small", pqtest.load("cfg4_small")), ("cfg4_v2", pqtest.load("cfg4_v2")),
                   ("deep1", T._deep_file("1.0")), ("deep2", T._deep_file("2.0"))):
    of = O.File(data)
    f, b, ids = T._gpu_nested_all(ctx, data)
    b.debug_counters(reset=True)
    for _ in range(2):  # the benchmark's pattern: decodes back to back, then one sync
        b.decode()
    assert b.sync() is None, name
    c = b.debug_counters(reset=True)
    torn += int(c[20]) & ((1 << 40) - 1)  # (nested.hip: slot 20, the guard's count in bits 40 and up)
    over += int(c[20]) >> 40
    for (rg, col), cid in ids.items():
        r = b.result(cid)
        o = of.read_chunk(rg, col)
        pqtest.assert_chunk_equal(r, o, f"torn {name} rg{rg} col{col}")
        lnd, ld, md = T._levels_of(data, col)
        want_levels, want_elem = T.nested_ref(o.rep_levels, o.def_levels, md, lnd, ld)
        T._check_nested(r.nested, r.element_validity, want_levels, want_elem, f"torn {name} rg{rg} col{col}")
    b.close()
print("TORN", torn, "OVER", over)
"""


@pytest.mark.gpu
def test_gpu_lookback_torn_publish():
    """k_nest_tile's look-back with the torn state made certain (diagnostic library, PQ_ABLATE bit 26:
    every tile publishes its counter words one at a time, in reverse order, ~27 us apart, nested.hip
    nest_publish). A successor then finds predecessors whose words are partly aggregates and partly
    inclusive prefixes (counted in debug slot 20) and must read them again rather than sum them: every
    nested array equals the oracle's on cfg4_small, cfg4_v2 and the two-list-level documents, and the
    prefix guard (a prefix past the chunk's slots; slot 20's high bits) never fires."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    diag = os.path.join(root, "parquet-go-1_amd", "lib", "libpqgpu_diag.so")
    assert os.path.exists(diag), "make -C parquet-go-1_amd diag"
    env = dict(os.environ, PQGPU_LIB=diag, PQ_ABLATE=str(1 << 26), PQ_DEBUG_STAMPS="1", PQ_NEST_FUSED="1",
               PQ_NEST_TCOUNT="0")
    tests = os.path.dirname(os.path.abspath(__file__))
    r = subprocess.run([sys.executable, "-c", TORN_SCRIPT, tests, os.path.join(root, "parquet-go-1_amd"),
                        os.path.join(root, "oracle")], env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("TORN")][-1].split()
    torn, over = int(line[1]), int(line[3])
    print(f"torn predecessors re-read: {torn}, guard fired: {over}")
    assert torn > 0, "the injection produced no torn state: the test would prove nothing"
    assert over == 0
