"""SNAPPY data pages decompressed on the GPU (k_snappy; compress.go:42-48,
:102-123; golang/snappy v0.0.1 decode_other.go — parity unpinned beyond the snappy block format
and pyarrow's codec).

Blocks are written by tools/rawpq.py's greedy encoder (checked here against pyarrow's snappy
codec) so that every element encoding occurs: literals with 0-4 length bytes, copies with 1-,
2- and 4-byte offsets, overlapping copies (offset < length), and offsets past the kernel's
LDS ring (16 KiB) and past 64 KiB. Corrupt blocks cover every ErrCorrupt condition of the
decoder, in the part of a page the host planner reads and in the part only the GPU reads, and
the reference's error order across pages (readPages decompresses page by page before any value
is decoded). The GPU must equal the oracle: values bit for bit, errors as (class, page)."""
import os
import sys
import zlib

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import rawpq  # noqa: E402

import pqtest  # noqa: E402
import py_oracle as O  # noqa: E402


def _data(kind, nbytes, rng):
    if kind == "random":  # incompressible: long literals
        return bytes(rng.integers(0, 256, nbytes, dtype=np.uint8))
    if kind == "smallint":  # int64 values < 16: short copies everywhere, overlapping runs
        return rng.integers(0, 16, nbytes // 8, dtype=np.int64).tobytes()
    if kind == "far":  # a 40 000-byte random period: copies reach past the ring (16 KiB)
        base = bytes(rng.integers(0, 256, 40_000, dtype=np.uint8))
        return (base * (nbytes // 40_000 + 1))[:nbytes]
    if kind == "far64k":  # 70 000-byte period: copy-4 offsets past 64 KiB
        base = bytes(rng.integers(0, 256, 70_000, dtype=np.uint8))
        return (base * (nbytes // 70_000 + 1))[:nbytes]
    raise ValueError(kind)


def _int64_file(pages, optional=False, v2=False, compress=None, encodings=None, rgs=1):
    """One INT64 column; pages = [(values bytes, num_slots, def level bytes or b"", num_nulls)]."""
    comp = compress or (lambda b: rawpq.snappy_compress(b))
    ps = []
    for k, (vals, ns, defs, nulls) in enumerate(pages):
        enc = (encodings or {}).get(k, "PLAIN")
        if v2:
            ps.append(rawpq.page_v2c(vals, ns, nulls, ns, enc, defs, comp))
        else:
            ps.append(rawpq.page_v1c(vals, ns, enc, defs, comp))
    n = sum(p[1] for p in pages)
    per = len(ps) // rgs
    groups = []
    for g in range(rgs):
        sl = slice(g * per, (g + 1) * per if g < rgs - 1 else len(ps))
        ns = sum(p[1] for p in pages[sl])
        groups.append((ns, [ps[sl]], [ns]))
    assert sum(g[0] for g in groups) == n
    return rawpq.write_file([("a", "INT64", optional)], groups, codec=1)


def _plain_pages(kind, sizes, seed, optional=False):
    rng = np.random.default_rng(seed)
    out = []
    for nb in sizes:
        raw = _data(kind, nb * 8, rng)
        nv = len(raw) // 8
        if not optional:
            out.append((raw[:nv * 8], nv, b"", 0))
            continue
        ns = nv + nv // 9 + 1
        valid = np.ones(ns, bool)
        valid[rng.choice(ns, ns - nv, replace=False)] = False
        defs = rawpq.hybrid_bitpacked([int(x) for x in valid], 1)
        out.append((raw[:nv * 8], ns, defs, ns - nv))
    return out


def _compare(gpu, data, where, rg=0):
    import pqgpu
    try:
        orc = O.File(data).read_chunk(rg, 0)
    except O.OracleError as r:
        assert isinstance(gpu, pqgpu.DecodeError), f"{where}: oracle error {r} but GPU decoded"
        assert (gpu.code, gpu.page) == (r.code, r.page), f"{where}: {gpu} vs {r}"
        return
    assert not isinstance(gpu, pqgpu.DecodeError), f"{where}: GPU error {gpu}"
    pqtest.assert_chunk_equal(gpu, orc, where)


def _gpu(ctx, data, rgs=(0,)):
    import pqgpu
    f = pqgpu.File(data)
    b = pqgpu.Batch(ctx)
    ids = [b.add_file_chunk(f, rg, 0) for rg in rgs]
    b.decode()
    b.sync()
    out = [e or b.status(cid) or b.result(cid) for cid, e in ids]
    b.close()
    return out


# ------------------------------------------------------------------ valid blocks
SIZES = [1, 7, 1000, 20_000, 131_072, 300_000]  # values per page (8 B each): up to 2.4 MB pages
VALID = {
    "random_v1": dict(kind="random"),
    "smallint_v1": dict(kind="smallint"),
    "far_v1": dict(kind="far"),
    "far64k_v1": dict(kind="far64k"),
    "smallint_opt_v1": dict(kind="smallint", optional=True),
    "random_opt_v2": dict(kind="random", optional=True, v2=True),
    "far_opt_v2": dict(kind="far", optional=True, v2=True),
    "mixed_kinds_v1": dict(kind="smallint", varied=True),
    "mixed_kinds_opt_v2": dict(kind="far", optional=True, v2=True, varied=True),
}


def _valid_file(name):
    c = VALID[name]
    pages = _plain_pages(c["kind"], SIZES, seed=zlib.crc32(name.encode()) % 1000, optional=c.get("optional", False))
    comp = None
    if c.get("varied"):
        rng = np.random.default_rng(5)
        comp = lambda b: rawpq.snappy_compress(b, rng)  # noqa: E731
    return _int64_file(pages, c.get("optional", False), c.get("v2", False), comp), pages


def test_encoder_matches_pyarrow_codec():
    pa = pytest.importorskip("pyarrow")
    codec = pa.Codec("snappy")
    rng = np.random.default_rng(3)
    for kind in ("random", "smallint", "far", "far64k"):
        d = _data(kind, 150_000, rng)
        for r in (None, np.random.default_rng(4)):
            z = rawpq.snappy_compress(d, r)
            assert codec.decompress(z, decompressed_size=len(d)).to_pybytes() == d
        # and the oracle's decoder on pyarrow's own blocks (through a page)
        d8 = d[:len(d) // 8 * 8]
        f = _int64_file([(d8, len(d8) // 8, b"", 0)], compress=lambda b: codec.compress(b, asbytes=True))
        got = O.File(f).read_chunk(0, 0)
        np.testing.assert_array_equal(np.asarray(pqtest.oracle_values(got)), np.frombuffer(d8, np.int64))


@pytest.mark.parametrize("name", sorted(VALID))
def test_oracle_valid(name):
    data, pages = _valid_file(name)
    got = O.File(data).read_chunk(0, 0)
    expect = np.concatenate([np.frombuffer(vals, np.int64) for vals, *_ in pages])
    np.testing.assert_array_equal(np.asarray(pqtest.oracle_values(got)), expect)


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(VALID))
def test_gpu_valid(gpu_ctx, name):
    data, _ = _valid_file(name)
    _compare(_gpu(gpu_ctx, data)[0], data, name)


@pytest.mark.gpu
def test_gpu_delta_pages(gpu_ctx):
    """DELTA pages: the host reads the block header from the decoded head of the block."""
    rng = np.random.default_rng(9)
    pages_vals = [rawpq.random_walk(rng, n, 12) for n in (100, 5000, 70_000)]
    ps = [rawpq.page_v1c(rawpq.delta_encode(v, 256, 4, 64), len(v), "DELTA_BINARY_PACKED", b"",
                         rawpq.snappy_compress) for v in pages_vals]
    n = sum(len(v) for v in pages_vals)
    data = rawpq.write_file([("a", "INT64", False)], [(n, [ps], [n])], codec=1)
    _compare(_gpu(gpu_ctx, data)[0], data, "delta")


@pytest.mark.gpu
def test_gpu_host_snappy_switch(gpu_ctx, monkeypatch):
    """PQ_HOST_SNAPPY=1 (host decompression) and the device path give the same chunk."""
    data, _ = _valid_file("far_opt_v2")
    dev = _gpu(gpu_ctx, data)[0]
    monkeypatch.setenv("PQ_HOST_SNAPPY", "1")
    host = _gpu(gpu_ctx, data)[0]
    orc = O.File(data).read_chunk(0, 0)
    pqtest.assert_chunk_equal(dev, orc, "device")
    pqtest.assert_chunk_equal(host, orc, "host")


# ------------------------------------------------------------------ corrupt blocks
def _elements(vals, rng=None):
    """The element list of a valid block (re-parsed from the encoder's output)."""
    z = rawpq.snappy_compress(vals, rng)
    k = 0
    while z[k] & 0x80:
        k += 1
    k += 1
    els = []
    while k < len(z):
        t = z[k]
        if t & 3 == 0:
            x = t >> 2
            h = 1 if x < 60 else x - 58
            ln = (x if x < 60 else int.from_bytes(z[k + 1:k + h], "little")) + 1
            size = h + ln
        else:
            size = {1: 2, 2: 3, 3: 5}[t & 3]
        els.append(z[k:k + size])
        k += size
    return els


def _bad_block(vals, how):
    """A block for `vals` (its length in the preamble) broken in the given way."""
    els = _elements(vals)
    n = len(vals)
    lits = [i for i, e in enumerate(els) if e[0] & 3 == 0]
    cps = [i for i, e in enumerate(els) if e[0] & 3 != 0]
    tail = len(els) * 3 // 4  # past the head the host reads
    if how.startswith("head_"):
        tail = 0
        how = how[5:]
    if how == "offset_zero":
        i = next((i for i in cps if i >= tail), cps[-1])
        ln = {1: 4 + ((els[i][0] >> 2) & 7), 2: 1 + (els[i][0] >> 2), 3: 1 + (els[i][0] >> 2)}[els[i][0] & 3]
        els[i] = rawpq.sn_copy(0, max(ln, 1), 2 if ln > 11 else 4)
    elif how == "offset_before_start":
        i = next((i for i in cps if i >= tail), cps[-1])
        d = sum(_out_len(e) for e in els[:i])
        els[i] = rawpq.sn_copy(d + 1, 4, 4)
    elif how == "literal_past_end":
        i = lits[-1]
        els = els[:i + 1]
        els[i] = els[i][:-1]  # the literal's last byte is missing
    elif how == "copy_past_dlen":
        i = cps[-1]
        els = els[:i + 1]
        e = els[i]
        d = sum(_out_len(x) for x in els[:i])
        off = _copy_off(e)
        els[i] = rawpq.sn_copy(off, min(64, n - d + 1), 4)
    elif how == "trailing_element":
        els.append(rawpq.sn_literal(b"x"))
    elif how == "short_output":
        els = els[:-1]
    elif how == "truncated_header":
        els = els[:-1] + [bytes([3 | (3 << 2), 1])]
    else:
        raise ValueError(how)
    return rawpq.snappy_block(n, els)


def _out_len(e):
    t = e[0]
    if t & 3 == 0:
        x = t >> 2
        h = 1 if x < 60 else x - 58
        return (x if x < 60 else int.from_bytes(e[1:h], "little")) + 1
    return {1: 4 + ((t >> 2) & 7), 2: 1 + (t >> 2), 3: 1 + (t >> 2)}[t & 3]


def _copy_off(e):
    t = e[0]
    if t & 3 == 1:
        return ((t & 0xE0) << 3) | e[1]
    return int.from_bytes(e[1:3] if t & 3 == 2 else e[1:5], "little")


HOWS = ["offset_zero", "offset_before_start", "literal_past_end", "copy_past_dlen", "trailing_element",
        "short_output", "truncated_header", "head_offset_zero", "head_offset_before_start"]


def _bad_file(how, page, v2=False, delta=False):
    """Three pages of compressible INT64 values; `page` gets the broken block."""
    rng = np.random.default_rng(11)
    pages = _plain_pages("smallint", [4000, 4000, 4000], 13, optional=v2)
    encs = {}
    if delta:  # DELTA values: the planner reads the block header from the head of the block
        pv = [rawpq.random_walk(rng, 4000, 6) for _ in range(3)]
        pages = [(rawpq.delta_encode(v, 128, 4, 64), 4000, b"", 0) for v in pv]
        encs = {k: "DELTA_BINARY_PACKED" for k in range(3)}

    def comp(b):  # pages are compressed in order
        out = _bad_block(b, how) if comp.k == page else rawpq.snappy_compress(b)
        comp.k += 1
        return out
    comp.k = 0
    return _int64_file(pages, optional=v2, v2=v2, compress=comp, encodings=encs)


BAD = [(how, page, v2, delta) for how in HOWS for page in (0, 2) for v2 in (False, True) for delta in (False,)]
BAD += [(how, 1, False, True) for how in ("head_offset_zero", "offset_zero", "short_output")]


@pytest.mark.parametrize("how,page,v2,delta", BAD)
def test_oracle_corrupt(how, page, v2, delta):
    data = _bad_file(how, page, v2, delta)
    with pytest.raises(O.OracleError) as ei:
        O.File(data).read_chunk(0, 0)
    assert (ei.value.code, ei.value.page) == (7, page), (how, ei.value)


@pytest.mark.gpu
@pytest.mark.parametrize("how,page,v2,delta", BAD)
def test_gpu_corrupt(gpu_ctx, how, page, v2, delta):
    data = _bad_file(how, page, v2, delta)
    _compare(_gpu(gpu_ctx, data)[0], data, f"{how} page {page} v2={v2} delta={delta}")


def _order_file():
    """Page 0: corrupt block tail (found by k_snappy); page 2: an unsupported encoding (found by
    the host planner). The reference decompresses page 0 first: DECOMPRESS at page 0."""
    pages = _plain_pages("smallint", [3000, 3000, 3000], 17)

    def comp(b):
        comp.k += 1
        return _bad_block(b, "short_output") if comp.k == 1 else rawpq.snappy_compress(b)
    comp.k = 0
    return _int64_file(pages, compress=comp, encodings={2: "RLE"})


def test_oracle_error_order():
    with pytest.raises(O.OracleError) as ei:
        O.File(_order_file()).read_chunk(0, 0)
    assert (ei.value.code, ei.value.page) == (7, 0)


def test_host_error_order():
    """The planner finds page 2's error first; the staged page-0 block is checked before it is
    reported (error path only), so the plan-only batch already reports page 0."""
    import pqgpu
    b = pqgpu.Batch(None)
    _, e = b.add_file_chunk(pqgpu.File(_order_file()), 0, 0)
    assert e is not None and (e.code, e.page) == (7, 0)
    b.close()


@pytest.mark.gpu
def test_gpu_error_order(gpu_ctx):
    data = _order_file()
    _compare(_gpu(gpu_ctx, data)[0], data, "order")


@pytest.mark.gpu
def test_gpu_corrupt_chunk_isolated(gpu_ctx):
    """A corrupt page fails only its own chunk: the other row group's chunk in the batch decodes."""
    pages = _plain_pages("smallint", [3000, 3000, 3000, 3000], 19)

    def comp(b):
        comp.k += 1
        return _bad_block(b, "offset_zero") if comp.k == 2 else rawpq.snappy_compress(b)
    comp.k = 0
    data = _int64_file(pages, compress=comp, rgs=2)
    got = _gpu(gpu_ctx, data, rgs=(0, 1))
    _compare(got[0], data, "rg0", rg=0)
    _compare(got[1], data, "rg1", rg=1)


def test_preamble_mismatch_host():
    """A preamble that disagrees with the page header is decoded on the host (reference error)."""
    pages = _plain_pages("smallint", [1000], 23)
    vals = pages[0][0]
    z = rawpq.snappy_compress(vals)
    bad = rawpq.uvar(len(vals) + 8) + z[len(rawpq.uvar(len(vals))):]
    data = _int64_file(pages, compress=lambda b: bad)
    with pytest.raises(O.OracleError) as ei:
        O.File(data).read_chunk(0, 0)
    assert (ei.value.code, ei.value.page) == (7, 0)
    import pqgpu
    b = pqgpu.Batch(None)
    cid, e = b.add_file_chunk(pqgpu.File(data), 0, 0)
    assert e is not None and (e.code, e.page) == (7, 0)
    b.close()


def _pyarrow_snappy_file(kind, rows=3 * 65536 + 777):
    """pyarrow (Arrow C++ snappy) V1 SNAPPY pages of 65,536 rows: the bench's page shape."""
    pa = pytest.importorskip("pyarrow")
    import io
    import pyarrow.parquet as pq
    rng = np.random.default_rng(11)
    if kind == "double_opt":  # def-level bitmap (short elements) + 64 KiB literals (direct path)
        col = pa.array(rng.random(rows), mask=rng.random(rows) < 0.1)
    elif kind == "int64_small":  # copies every few bytes, ring wrap-around, HBM flushes
        col = pa.array(rng.integers(0, 16, rows).astype(np.int64))
    else:  # "int64_small_opt"
        col = pa.array(rng.integers(0, 16, rows).astype(np.int64), mask=rng.random(rows) < 0.3)
    bio = io.BytesIO()
    pq.write_table(pa.table({"c": col}), bio, use_dictionary=False, data_page_version="1.0",
                   compression="SNAPPY", column_encoding={"c": "PLAIN"}, max_rows_per_page=65536,
                   write_statistics=False)
    return bio.getvalue()


@pytest.mark.parametrize("kind", ["double_opt", "int64_small", "int64_small_opt"])
def test_oracle_pyarrow_pages(kind):
    data = _pyarrow_snappy_file(kind)
    got = O.File(data).read_chunk(0, 0)
    assert got.num_values > 0


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["double_opt", "int64_small", "int64_small_opt"])
def test_gpu_pyarrow_pages(gpu_ctx, kind):
    data = _pyarrow_snappy_file(kind)
    _compare(_gpu(gpu_ctx, data)[0], data, kind)


# ------------------------------------------------------------------ direct output (SnappyJob::lead)
def _typed_file(typ, width, counts, seed, extra=None):
    """One REQUIRED column of `typ` (PLAIN, SNAPPY V1): pages of `counts` values; extra[k] = bytes
    appended to page k's body (or removed, when negative) so its decoded length is not count x width."""
    rng = np.random.default_rng(seed)
    ps = []
    for k, nv in enumerate(counts):
        body = bytes(rng.integers(0, 256, nv * width, dtype=np.uint8)) if k % 2 else \
            rng.integers(0, 7, nv * width, dtype=np.uint8).tobytes()
        d = (extra or {}).get(k, 0)
        body = body + bytes(range(d)) if d > 0 else body[:len(body) + d]
        ps.append(rawpq.page_v1c(body, nv, "PLAIN", b"", lambda b: rawpq.snappy_compress(b)))
    n = sum(counts)
    return rawpq.write_file([("a", typ, False)], [(n, [ps], [n])], codec=1)


DIRECT = {  # value bases not 16-B aligned in every combination, one-value and odd-length pages
    "int32": ("INT32", 4, [1, 3, 2, 5, 1000, 20_001, 7]),
    "float": ("FLOAT", 4, [6, 1, 4097, 3]),
    "int96": ("INT96", 12, [1, 2, 3, 333, 5000, 1]),
    "int64": ("INT64", 8, [1, 1, 1, 7, 9, 65_537]),
}


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(DIRECT))
def test_gpu_direct_values(gpu_ctx, name):
    """REQUIRED PLAIN pages that k_snappy writes straight into the values array (no k_values copy):
    neighbouring pages share 16-B pieces at every alignment; the result equals the oracle, with the
    direct path on and off."""
    typ, w, counts = DIRECT[name]
    data = _typed_file(typ, w, counts, seed=len(name))
    g = _gpu(gpu_ctx, data)[0]
    _compare(g, data, f"direct {name}")


@pytest.mark.gpu
@pytest.mark.parametrize("delta", [-1, -4, 3, 8])
def test_gpu_direct_values_size_mismatch(gpu_ctx, delta):
    """A page whose decoded length is not num_values x width takes the copy path and keeps the
    reference's outcome (a short body: EOF / ErrUnexpectedEOF at the first missing value; a longer
    one: the extra bytes are ignored)."""
    data = _typed_file("INT64", 8, [5, 11, 3], seed=3, extra={1: delta})
    _compare(_gpu(gpu_ctx, data)[0], data, f"mismatch {delta}")


@pytest.mark.gpu
def test_gpu_direct_switch(gpu_ctx, monkeypatch):
    """PQ_SNAPPY_DIRECT=0 (every page through k_values) gives the same values."""
    data = _typed_file("INT32", 4, DIRECT["int32"][2], seed=9)
    a = _gpu(gpu_ctx, data)[0]
    monkeypatch.setenv("PQ_SNAPPY_DIRECT", "0")
    b = _gpu(gpu_ctx, data)[0]
    assert np.asarray(a.values_raw).tobytes() == np.asarray(b.values_raw).tobytes()


@pytest.mark.gpu
@pytest.mark.parametrize("groups", ["1", "2", "3", "8"])
def test_gpu_column_groups(gpu_ctx, monkeypatch, groups):
    """The column-group pipeline (host.cpp n_groups: group g's run scan, dictionary tiles and DELTA
    pages start when group g's SNAPPY launch is done) on the 64-column cfg5 replica, with 1 (off) to 8
    groups: every chunk equals the oracle."""
    import pqgpu
    monkeypatch.setenv("PQ_SNAPPY_GROUPS", groups)
    data = pqtest.load("cfg5_small")
    f = pqgpu.File(data)
    gpu = {}
    for rg in range(f.num_row_groups):  # one batch per row group: each batch is cut into groups
        b = pqgpu.Batch(gpu_ctx)
        b.kernel_timing(True)
        ids = {col: b.add_file_chunk(f, rg, col)[0] for col in range(f.num_columns)}
        b.decode()
        b.sync()
        # the pipeline really ran: one SNAPPY launch per group
        assert b.kernel_times()["k_snappy"][1] == min(int(groups), f.num_columns), b.kernel_times()
        for col, cid in ids.items():
            e = b.status(cid)
            gpu[(rg, col)] = e if e is not None else b.result(cid)
        b.close()
    for rg, col, r in pqtest.oracle_decode(data):
        pqtest.assert_chunk_equal(gpu[(rg, col)], r, f"groups {groups} rg{rg} col{col}")
