"""The reference's own level goldens (Dremel paper and Twitter examples), transcribed from
data_store_test.go: TestOneColumnOptional (:47-73), TestOneColumnRepeated (:75-102),
TestComplex (:227-345) and TestTwitterBlog (:346-390). For every column the test lists
maxD/maxR, the non-null values and the exact definition/repetition level sequences.

Those levels are written here as the reference writer writes them (one bit-packed hybrid run
per stream at bits.Len16(max), PLAIN values, V1 and V2 pages; tools/rawpq.py) into one file
per document. The oracle must read back exactly the transcribed levels and values (this pins
the oracle's level decoding to the reference's tests), and the GPU must equal the oracle."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import rawpq  # noqa: E402

import py_oracle as O  # noqa: E402

G, L = rawpq.schema_group, rawpq.schema_leaf

# name -> (schema elements, [(path, maxD, maxR, values, dL, rL)], number of records)
DOCS = {
    # TestComplex: the Dremel paper document pair (data_store_test.go:227-345)
    "dremel": (
        [[(4, rawpq.BIN, "schema"), (5, rawpq.I32, 3)],
         L("DocId", "INT32", "REQUIRED"),
         G("Links", "OPTIONAL", 2), L("Backward", "INT32", "REPEATED"), L("Forward", "INT32", "REPEATED"),
         G("Name", "REPEATED", 2), G("Language", "REPEATED", 2), L("Code", "INT32", "REQUIRED"),
         L("Country", "INT32", "OPTIONAL"), L("URL", "INT32", "OPTIONAL")],
        [("DocId", 0, 0, [10, 20], [0, 0], [0, 0]),
         ("Links.Backward", 2, 1, [10, 30], [1, 2, 2], [0, 0, 1]),
         ("Links.Forward", 2, 1, [20, 40, 60, 80], [2, 2, 2, 2], [0, 1, 1, 0]),
         ("Name.Language.Code", 2, 2, [1, 2, 3], [2, 2, 1, 2, 1], [0, 2, 1, 1, 0]),
         ("Name.Language.Country", 3, 2, [100, 101], [3, 2, 1, 3, 1], [0, 2, 1, 1, 0]),
         ("Name.URL", 2, 1, [10, 11, 12], [2, 2, 1, 2], [0, 1, 1, 0])],
        2),
    # TestTwitterBlog (:346-390)
    "twitter": (
        [[(4, rawpq.BIN, "schema"), (5, rawpq.I32, 1)],
         G("level1", "REPEATED", 1), L("level2", "INT32", "REPEATED")],
        [("level1.level2", 2, 2, list(range(1, 11)), [2] * 10, [0, 2, 2, 1, 2, 2, 2, 0, 1, 2])],
        2),
    # TestOneColumnRepeated (:75-102) and TestOneColumnOptional (:47-73)
    "one_repeated": (
        [[(4, rawpq.BIN, "schema"), (5, rawpq.I32, 1)], L("DocID", "INT32", "REPEATED")],
        [("DocID", 1, 1, [10, 20], [1, 1, 0], [0, 1, 0])],
        2),
    "one_optional": (
        [[(4, rawpq.BIN, "schema"), (5, rawpq.I32, 1)], L("DocID", "INT32", "OPTIONAL")],
        [("DocID", 1, 0, [10], [1, 0], [0, 0])],
        2),
}


# Not reference documents: inputs for other tests, built the same way.
EXTRA = {
    # a MAP whose key and value leaves disagree about the entries of each map (record 1: two keys but
    # one value entry; record 2: one key, two value entries): test_struct's shared-ancestor check
    "map_mismatch": (
        [[(4, rawpq.BIN, "schema"), (5, rawpq.I32, 1)],
         G("m", "OPTIONAL", 1), G("key_value", "REPEATED", 2), L("key", "INT32", "REQUIRED"),
         L("value", "INT32", "OPTIONAL")],
        [("m.key_value.key", 2, 1, [1, 2, 3], [2, 2, 2], [0, 1, 0]),
         ("m.key_value.value", 3, 1, [10, 20], [3, 3, 2], [0, 0, 1])],
        2),
}


def build(name, v2=False, crc=False):
    schema, cols, nrec = DOCS[name] if name in DOCS else EXTRA[name]
    chunks = []
    for path, md, mr, vals, dl, rl in cols:
        body = rawpq.plain_encode("INT32", vals)
        if v2:
            nulls = sum(1 for d in dl if d < md)
            p = rawpq.data_page_v2_ref(len(dl), nulls, nrec, "PLAIN", body, dl, md, rl, mr, crc=crc)
        else:
            p = rawpq.data_page_v1_ref(len(dl), "PLAIN", body, dl, md, rl, mr, crc=crc)
        chunks.append(([p], len(dl), False))
    return rawpq.write_file_schema(schema, [(c[0], "INT32") for c in cols], [(nrec, chunks)])


CASES = [(n, v2) for n in sorted(DOCS) for v2 in (False, True)]


@pytest.mark.parametrize("name,v2", CASES)
def test_oracle_reads_reference_levels(name, v2):
    """The oracle reproduces the reference test's maxD/maxR, values, dL and rL."""
    data = build(name, v2, crc=True)
    f = O.File(data)
    _, cols, _ = DOCS[name]
    assert f.num_columns == len(cols)
    for c, (path, md, mr, vals, dl, rl) in enumerate(cols):
        info = f.column_info(c)
        assert info.path.decode() == path
        assert (info.max_def, info.max_rep) == (md, mr), path
        r = f.read_chunk(0, c, validate_crc=True)
        assert list(r.def_levels) == dl, path
        assert list(r.rep_levels) == rl, path
        assert list(np.asarray(r.values).view(np.int32)) == vals, path


@pytest.mark.parametrize("name,v2", CASES)
def test_host_schema_levels(name, v2):
    """libpqgpu's footer/schema walk gives the reference's maxD/maxR (schema.go:893-990)."""
    import pqgpu
    f = pqgpu.File(build(name, v2))
    _, cols, _ = DOCS[name]
    for c, (path, md, mr, *_r) in enumerate(cols):
        ci = f.column(c)
        assert (ci.path.decode(), ci.max_def, ci.max_rep) == (path, md, mr)


@pytest.mark.gpu
@pytest.mark.parametrize("name,v2", CASES)
def test_gpu_reference_levels(gpu_ctx, name, v2):
    import pqgpu
    import pqtest
    data = build(name, v2, crc=True)
    f = pqgpu.File(data)
    of = O.File(data)
    b = pqgpu.Batch(gpu_ctx)
    _, cols, _ = DOCS[name]
    ids = [b.add_file_chunk(f, 0, c, validate_crc=True)[0] for c in range(len(cols))]
    b.decode()
    assert b.sync() is None
    for c, cid in enumerate(ids):
        path, md, mr, vals, dl, rl = cols[c]
        g = b.result(cid)
        pqtest.assert_chunk_equal(g, of.read_chunk(0, c), f"{name} {path}")
        assert list(g.dLevels) == dl and list(g.rLevels) == rl, path
    b.close()
