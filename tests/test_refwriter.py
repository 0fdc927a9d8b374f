"""Streams in the reference writer's own layout, which pyarrow never
produces: every hybrid stream (definition/repetition levels and dictionary indices) is ONE
bit-packed run (hybrid_encoder.go:55-70), dictionary index width is bits.Len(len(dict)) — 9 bits
for 256 entries (page_v1.go:185, page_v2.go:200) — and DELTA streams use 128-value blocks of
4 miniblocks. The generator knows every value; the oracle must return them, and the GPU must
equal the oracle. Also: page CRCs (WithCRC32Validation, chunk_reader.go:173-177)."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import rawpq  # noqa: E402

import pqtest  # noqa: E402
import py_oracle as O  # noqa: E402

PAGE_ROWS = [1000, 4096, 1, 8, 7, 30000]


def _words(rng, k):
    out = set()
    while len(out) < k:
        out.add(bytes(rng.integers(97, 123, int(rng.integers(0, 20)), dtype=np.uint8)))
    return sorted(out)


def build(v2, dict_size=256, seed=0, crc=False):
    """Columns: i32 OPTIONAL RLE_DICTIONARY (dict_size entries), s BYTE_ARRAY OPTIONAL
    RLE_DICTIONARY (300 entries), d INT64 OPTIONAL DELTA_BINARY_PACKED 128x4, p DOUBLE REQUIRED
    PLAIN. Pages of PAGE_ROWS rows. Returns (file bytes, expected {col: (values, def levels)})."""
    rng = np.random.default_rng(100 + seed)
    n = sum(PAGE_ROWS)
    d32 = rng.integers(-2**31, 2**31 - 1, dict_size, dtype=np.int64).astype(np.int32)
    vocab = _words(rng, 300)
    cols = {
        "i32": (rng.integers(0, dict_size, n), rng.random(n) < 0.2),
        "s": (rng.integers(0, 300, n), rng.random(n) < 0.1),
        "d": (np.cumsum(rng.integers(-5000, 70000, n)).astype(np.int64), rng.random(n) < 0.15),
        "p": (rng.random(n), np.zeros(n, bool)),
    }
    # DELTA pages the reference can read back: >= 1 value and not 1 mod 128 (App. A Q1)
    at = 0
    for pr in PAGE_ROWS:
        m = cols["d"][1][at:at + pr]
        m[0] = False
        if (~m).sum() > 1 and (~m).sum() % 128 == 1:
            m[np.flatnonzero(~m)[-1]] = True
        at += pr
    expect, chunks = {}, []
    for name, (vals, nulls) in cols.items():
        dl = (~nulls).astype(int).tolist()
        md = 0 if name == "p" else 1
        pages = []
        if name == "i32":
            pages.append(rawpq.dict_page_ref("INT32", d32, crc=crc))
        if name == "s":
            pages.append(rawpq.dict_page_ref("BYTE_ARRAY", vocab, crc=crc))
        at = 0
        for pr in PAGE_ROWS:
            sl = slice(at, at + pr)
            at += pr
            nn = vals[sl][~nulls[sl]]
            if name in ("i32", "s"):
                enc, body = "RLE_DICTIONARY", rawpq.dict_values_section(nn, dict_size if name == "i32" else 300)
            elif name == "d":
                enc, body = "DELTA_BINARY_PACKED", rawpq.delta_encode([int(x) for x in nn], 128, 4, 64,
                                                                      ref_single=True)
            else:
                enc, body = "PLAIN", rawpq.plain_encode("DOUBLE", nn)
            pdl = dl[sl]
            if v2:
                pages.append(rawpq.data_page_v2_ref(pr, pr - len(nn), pr, enc, body, pdl, md, crc=crc))
            else:
                pages.append(rawpq.data_page_v1_ref(pr, enc, body, pdl, md, crc=crc))
        nnv = vals[~nulls]
        if name == "i32":
            ev = d32[nnv]
        elif name == "s":
            ev = [vocab[i] for i in nnv]
        elif name == "p":
            ev = nnv.view(np.uint64)
        else:
            ev = nnv
        expect[name] = (ev, np.array(dl) if md else np.zeros(n, int))
        chunks.append((pages, n, name in ("i32", "s")))
    schema = [[(4, rawpq.BIN, "schema"), (5, rawpq.I32, 4)], rawpq.schema_leaf("i32", "INT32", "OPTIONAL"),
              rawpq.schema_leaf("s", "BYTE_ARRAY", "OPTIONAL"), rawpq.schema_leaf("d", "INT64", "OPTIONAL"),
              rawpq.schema_leaf("p", "DOUBLE", "REQUIRED")]
    leaves = [("i32", "INT32"), ("s", "BYTE_ARRAY"), ("d", "INT64"), ("p", "DOUBLE")]
    return rawpq.write_file_schema(schema, leaves, [(n, chunks)]), expect


CASES = [(v2, ds) for v2 in (False, True) for ds in (256, 255, 1, 2, 65536)]


def _check_oracle(data, expect, crc=False):
    f = O.File(data)
    for c, name in enumerate(["i32", "s", "d", "p"]):
        r = f.read_chunk(0, c, validate_crc=crc)
        ev, dl = expect[name]
        np.testing.assert_array_equal(r.def_levels, dl, err_msg=name)
        got = pqtest.oracle_values(r)
        if name == "s":
            assert got == ev, name
        else:
            assert np.asarray(got).tobytes() == np.asarray(ev).tobytes(), name


@pytest.mark.parametrize("v2,dict_size", CASES)
def test_oracle_reference_style_streams(v2, dict_size):
    data, expect = build(v2, dict_size)
    _check_oracle(data, expect)


def test_reference_index_width():
    """bits.Len(len(dict)): 256 entries -> 9-bit indices (pyarrow would use 8)."""
    sec = rawpq.dict_values_section([0, 255], 256)
    assert sec[0] == 9 and sec[1] == 3  # one bit-packed run of one group


@pytest.mark.gpu
@pytest.mark.parametrize("v2,dict_size", CASES)
def test_gpu_reference_style_streams(gpu_ctx, v2, dict_size):
    import test_gpu_parity as P
    data, expect = build(v2, dict_size)
    gpu = P._gpu_decode(gpu_ctx, data)
    for rg, col, r in pqtest.oracle_decode(data):
        pqtest.assert_chunk_equal(gpu[(rg, col)], r, f"v2={v2} dict={dict_size} col{col}")


# ---------------------------------------------------------------- CRC32 validation


def test_oracle_crc():
    _check_oracle(*build(False, 256, crc=True), crc=True)
    good = pqtest.load("crc_v1")
    bad = pqtest.load("crc_v1_flipped")
    for rg, col, r in pqtest.oracle_decode(good):
        assert not isinstance(r, O.OracleError)
    f = O.File(bad)
    with pytest.raises(O.OracleError) as ei:
        f.read_chunk(0, 0, validate_crc=True)
    assert (ei.value.code, ei.value.page) == (6, 1)
    f.read_chunk(0, 0, validate_crc=False)  # without the option the flipped byte decodes


def test_host_crc_plan():
    """The host planner (readPages on the host) fails the flipped page exactly like the oracle."""
    import pqgpu
    f = pqgpu.File(pqtest.load("crc_v1_flipped"))
    b = pqgpu.Batch(None)
    cid, e = b.add_file_chunk(f, 0, 0, validate_crc=True)
    assert e is not None and (e.code, e.page) == (6, 1)
    cid, e = b.add_file_chunk(f, 0, 1, validate_crc=True)
    assert e is None
    b.close()
    b = pqgpu.Batch(None)
    assert b.add_file_chunk(f, 0, 0, validate_crc=False)[1] is None
    b.close()


@pytest.mark.gpu
def test_gpu_crc(gpu_ctx):
    import pqgpu
    for name in ("crc_v1", "crc_v1_flipped"):
        data = pqtest.load(name)
        f, of = pqgpu.File(data), O.File(data)
        for crc in (False, True):
            b = pqgpu.Batch(gpu_ctx)
            ids = [b.add_file_chunk(f, 0, c, validate_crc=crc)[0] for c in range(f.num_columns)]
            b.decode()
            b.sync()
            for c, cid in enumerate(ids):
                try:
                    r = of.read_chunk(0, c, validate_crc=crc)
                except O.OracleError as oe:
                    e = b.status(cid)
                    assert e is not None and (e.code, e.page) == (oe.code, oe.page), (name, crc, c)
                    continue
                pqtest.assert_chunk_equal(b.result(cid), r, f"{name} crc={crc} col{c}")
            b.close()
