"""GPU parity: every fixture decoded by the MI355X kernels (through the C ABI)
must equal the CPU oracle bit for bit — values, def/rep levels, validity,
byte-array offsets and payload, record offsets — and fail with the same
error class on the same page where the reference fails."""
import numpy as np
import pytest

import pqgpu
import pqtest
import py_oracle as O

pytestmark = pytest.mark.gpu


def _gpu_decode(ctx, data):
    f = pqgpu.File(data)
    b = pqgpu.Batch(ctx)
    ids = {}
    host_err = {}
    for rg in range(f.num_row_groups):
        for col in range(f.num_columns):
            cid, e = b.add_file_chunk(f, rg, col)
            ids[(rg, col)] = cid
            host_err[(rg, col)] = e
    b.decode()
    b.sync()
    out = {}
    for k, cid in ids.items():
        e = b.status(cid)
        out[k] = e if e is not None else b.result(cid)
    b.close()
    return out


@pytest.mark.parametrize("name", pqtest.ALL)
def test_fixture_parity(gpu_ctx, name):
    data = pqtest.load(name)
    try:
        orc = pqtest.oracle_decode(data)
    except O.OracleError:
        pytest.skip("footer-level error: covered by CPU tests")
    gpu = _gpu_decode(gpu_ctx, data)
    for rg, col, r in orc:
        g = gpu[(rg, col)]
        where = f"{name} rg{rg} col{col}"
        if isinstance(r, O.OracleError):
            assert isinstance(g, pqgpu.DecodeError), f"{where}: oracle error {r} but GPU decoded"
            assert (g.code, g.page) == (r.code, r.page), f"{where}: {g} vs {r}"
        else:
            assert not isinstance(g, pqgpu.DecodeError), f"{where}: GPU error {g}"
            pqtest.assert_chunk_equal(g, r, where)


@pytest.mark.parametrize("name", ["cfg1", "cfg1_full", "types_dict", "bad_dict_index", "cfg5_small", "edge_tiny_pages",
                                  "edge_nulls_v1", "edge_nulls_v2", "cfg4_small"])
def test_fixture_parity_paired_dict_tiles(gpu_ctx, name, monkeypatch):
    """Every dictionary tile pairing it can (PQ_DICT_PAIR=1: k_values_dict2, two tiles of a page
    per workgroup, host.cpp) must give the oracle's values, and its errors at the same page."""
    monkeypatch.setenv("PQ_DICT_PAIR", "1")
    test_fixture_parity(gpu_ctx, name)


@pytest.mark.parametrize("name,expected", sorted(pqtest.EXPECTED_ERRORS.items()))
def test_expected_errors(gpu_ctx, name, expected):
    gpu = _gpu_decode(gpu_ctx, pqtest.load(name))
    errs = [v for k, v in sorted(gpu.items()) if isinstance(v, pqgpu.DecodeError)]
    assert errs and (errs[0].code, errs[0].page) == expected, (name, errs[:1])


def test_must_not_crash_gpu(gpu_ctx):
    """The reference's fuzz regression images: the GPU path must return the oracle's result for
    every chunk — the same error class on the same page, or the same decoded bytes."""
    import os
    d = os.path.join(pqtest.GOLDEN, "must_not_crash")
    checked = 0
    for fn in sorted(os.listdir(d)):
        data = open(os.path.join(d, fn), "rb").read()
        try:
            orc = pqtest.oracle_decode(data)
        except O.OracleError as oe:
            with pytest.raises(pqgpu.DecodeError) as ei:
                pqgpu.File(data)
            assert ei.value.code == oe.code, (fn, ei.value, oe)
            continue
        gpu = _gpu_decode(gpu_ctx, data)
        for rg, col, r in orc:
            g = gpu[(rg, col)]
            where = f"{fn} rg{rg} col{col}"
            if isinstance(r, O.OracleError):
                assert isinstance(g, pqgpu.DecodeError), f"{where}: oracle error {r} but GPU decoded"
                assert (g.code, g.page) == (r.code, r.page), f"{where}: {g} vs {r}"
            else:
                assert not isinstance(g, pqgpu.DecodeError), f"{where}: GPU error {g}"
                pqtest.assert_chunk_equal(g, r, where)
            checked += 1
    assert checked > 0


def test_file_reader_mirror(gpu_ctx):
    """FileReader.ReadRowGroupData mirrors readRowGroupData for the selected columns."""
    data = pqtest.load("cfg2_v2_small")
    r = pqgpu.NewFileReader(data, "a", ctx=gpu_ctx)
    assert r.NumRowGroups() == 2
    cols = r.ReadRowGroupData(1)
    assert list(cols) == ["a"]
    orc = O.File(data).read_chunk(1, 0)
    pqtest.assert_chunk_equal(cols["a"], orc, "reader")


def test_speculative_and_serial_schedules_agree(gpu_ctx, monkeypatch):
    """V2 pages carry num_nulls, so values run concurrently with the level decode on header
    counts (host.cpp decode_impl, the default); PQ_SPEC=0 keeps the reference's serial order. Both must
    give the oracle's bytes, including on a file whose num_nulls header is wrong."""
    for name in ("cfg2_v2_small", "bad_v2_num_nulls", "edge_nulls_v2", "cfg4_v2"):
        data = pqtest.load(name)
        orc = pqtest.oracle_decode(data)
        for serial in ("0", "1"):
            monkeypatch.setenv("PQ_SPEC", "1" if serial == "0" else "0")
            gpu = _gpu_decode(gpu_ctx, data)
            for rg, col, r in orc:
                pqtest.assert_chunk_equal(gpu[(rg, col)], r, f"{name} serial={serial} rg{rg} col{col}")


@pytest.mark.parametrize("name", ["cfg2_v2_small", "cfg3_small", "cfg4_small", "cfg4_v2", "cfg5_small", "types_v2",
                                  "bad_dict_index"])
def test_one_stream_schedule_agrees(gpu_ctx, name, monkeypatch):
    """PQ_ONE_STREAM=1 runs every kernel of a decode on the batch stream (no DELTA / copy / side
    streams, the byte-array look-back instead of the pre-pass beside nested arrays): the profiling
    schedule must give the oracle's bytes, and its errors at the same page."""
    monkeypatch.setenv("PQ_ONE_STREAM", "1")
    test_fixture_parity(gpu_ctx, name)


def test_chunk_page_split(gpu_ctx):
    """pqgpu_batch_chunk_pages: page k of a chunk owns its header's num_values level slots and
    the non-null values its definition levels count, in order (data_store.go:236-260)."""
    for name in ("cfg2_v2_small", "edge_nulls_v1", "cfg4_small", "edge_tiny_pages"):
        data = pqtest.load(name)
        f = pqgpu.File(data)
        b = pqgpu.Batch(gpu_ctx)
        ids = [(rg, c, b.add_file_chunk(f, rg, c)[0]) for rg in range(f.num_row_groups) for c in range(f.num_columns)]
        b.decode()
        assert b.sync() is None
        for rg, c, cid in ids:
            r = b.result(cid)
            pg = b.pages(cid)
            assert pg[:, 1].sum() == r.num_slots and pg[:, 3].sum() == r.num_values
            assert (pg[:, 0] == np.concatenate([[0], np.cumsum(pg[:-1, 1])])).all()
            assert (pg[:, 2] == np.concatenate([[0], np.cumsum(pg[:-1, 3])])).all()
            dl = np.asarray(r.dLevels)
            for s0, sn, v0, vn in pg:  # values counted per page from the def levels (helpers.go:141-143)
                want = int((dl[s0:s0 + sn] == r.max_def).sum()) if r.max_def > 0 else sn
                assert vn == want, (name, rg, c)
        b.close()


@pytest.mark.parametrize("route", ["default", "gather"])
def test_repeated_decode_with_failed_byte_array_chunk(gpu_ctx, route, monkeypatch):
    """A batch decoded twice (the benchmark's pattern) whose first BYTE_ARRAY chunk fails on the
    device (dictionary index out of range, type_dict.go:52-54) and whose second decodes: the good
    chunk must be identical after both decodes, and the bad one must keep its error. Every
    k_ba_emit route of a 16/32-B slot dictionary (test_ba_classes.BA_ROUTES)."""
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(pqtest.GOLDEN), "..", "tools"))
    import rawpq
    import test_ba_classes
    test_ba_classes.set_route(monkeypatch, route)
    rng = np.random.default_rng(5)
    vocab = sorted({bytes(rng.integers(97, 123, int(rng.integers(1, 30)), dtype=np.uint8)) for _ in range(200)})
    n = 5000
    cols = []
    for bad in (True, False):
        idx = rng.integers(0, len(vocab), n)
        if bad:
            idx[3000] = len(vocab) + 3  # fits the 8-bit width, past the dictionary
        pages = [rawpq.dict_page_ref("BYTE_ARRAY", vocab),
                 rawpq.data_page_v1_ref(n, "RLE_DICTIONARY", rawpq.dict_values_section(idx, len(vocab)))]
        cols.append((pages, n, True))
    schema = [[(4, rawpq.BIN, "schema"), (5, rawpq.I32, 2)], rawpq.schema_leaf("bad", "BYTE_ARRAY", "REQUIRED"),
              rawpq.schema_leaf("good", "BYTE_ARRAY", "REQUIRED")]
    data = rawpq.write_file_schema(schema, [("bad", "BYTE_ARRAY"), ("good", "BYTE_ARRAY")], [(n, cols)])
    orc = pqtest.oracle_decode(data)
    assert isinstance(orc[0][2], O.OracleError) and orc[0][2].code == pqgpu.PQ_ERR_DICT_INDEX
    f = pqgpu.File(data)
    b = pqgpu.Batch(gpu_ctx)
    ids = [b.add_file_chunk(f, 0, c)[0] for c in range(2)]
    for _ in range(3):
        b.decode()
        e = b.sync()
        assert e is not None and (e.code, e.page) == (orc[0][2].code, orc[0][2].page)
        pqtest.assert_chunk_equal(b.result(ids[1]), orc[1][2], "good chunk")
    b.close()


def _cfg2_delta_corrupt(page=2):
    """cfg2_v2_small with the first miniblock width of column a's DELTA page `page` set to 70 (> 64:
    the reference's init() rejects it, deltabp_decoder.go:101-105)."""
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(pqtest.GOLDEN), "..", "tools"))
    import pqinspect
    buf = bytearray(pqtest.load("cfg2_v2_small"))
    ph, j = list(pqinspect.pages(bytes(buf), 0, 0))[page]
    assert ph[1] == 3 and ph[8][4] == 5  # DATA_PAGE_V2, DELTA_BINARY_PACKED
    p = j + ph[8][6] + ph[8][5]  # past the rep and def sections
    for _ in range(5):  # block size, miniblocks, count, first value, min delta
        _, p = pqinspect.uvar(buf, p)
    buf[p] = 70
    return bytes(buf)


@pytest.mark.parametrize("which", ["good", "delta_error", "level_error"])
def test_back_to_back_delta_major(gpu_ctx, which):
    """The DELTA-major schedule (host.cpp decode_impl: speculative V2 OPTIONAL DELTA + PLAIN, cfg2's
    shape) rotates two error-key buffers between consecutive decodes and defers the level stream's
    join. Three decodes queued back to back, then one sync (the benchmark's pattern), then decode +
    sync pairs: every chunk equals the oracle each time, and an error in a DELTA page or in a
    definition-level stream is reported with the reference's (code, page) every time."""
    data = {"good": lambda: pqtest.load("cfg2_v2_small"), "delta_error": _cfg2_delta_corrupt,
            "level_error": lambda: pqtest.load("bad_def_empty_run")}[which]()
    orc = pqtest.oracle_decode(data)
    bad = [(rg, col, r) for rg, col, r in orc if isinstance(r, O.OracleError)]
    assert bool(bad) == (which != "good"), bad
    f = pqgpu.File(data)
    b = pqgpu.Batch(gpu_ctx)
    ids = {(rg, col): b.add_file_chunk(f, rg, col)[0] for rg in range(f.num_row_groups) for col in range(f.num_columns)}
    for rounds in (3, 1, 1, 2, 1):
        for _ in range(rounds):
            b.decode()
        e = b.sync()
        assert (e is None) == (not bad), e
        for rg, col, r in orc:
            g = b.status(ids[(rg, col)])
            where = f"{which} x{rounds} rg{rg} col{col}"
            if isinstance(r, O.OracleError):
                assert g is not None and (g.code, g.page) == (r.code, r.page), (where, g, r)
            else:
                assert g is None, (where, g)
                pqtest.assert_chunk_equal(b.result(ids[(rg, col)]), r, where)
    b.close()


def _cfg1_run_corrupt(page=2, run=3):
    """cfg1 with run header `run` of dictionary data page `page` set to 0x00 (an RLE run of count 0:
    the reference's next() fails with "rle: empty RLE run", hybrid_decoder.go:123-125)."""
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(pqtest.GOLDEN), "..", "tools"))
    import pqinspect
    buf = bytearray(pqtest.load("cfg1"))
    ph, j = [(ph, j) for ph, j in pqinspect.pages(bytes(buf)) if ph[1] == 0][page]
    bw = buf[j]
    q = j + 1
    for _ in range(run):
        h, q2 = pqinspect.uvar(buf, q)
        q = q2 + ((h >> 1) * bw if h & 1 else (bw + 7) // 8)
    buf[q] = 0
    return bytes(buf)


@pytest.mark.parametrize("which", ["good", "dict_error", "run_error"])
def test_back_to_back_dict_only(gpu_ctx, which):
    """The dictionary-only schedule (host.cpp decode_impl: flat REQUIRED dictionary columns, cfg1's
    shape) puts only k_scan_runs and the dictionary launch on the stream per decode: the scan resets its
    pages' tile tables and the dictionary launch the next decode's error keys. Queued decodes, then
    decode + sync pairs: every chunk equals the oracle each time, and an index outside the dictionary
    (k_values_dict) or an empty run (k_scan_runs) is reported with the reference's (code, page)."""
    data = {"good": lambda: pqtest.load("cfg1"), "dict_error": lambda: pqtest.load("bad_dict_index"),
            "run_error": _cfg1_run_corrupt}[which]()
    orc = pqtest.oracle_decode(data)
    bad = [(rg, col, r) for rg, col, r in orc if isinstance(r, O.OracleError)]
    assert bool(bad) == (which != "good"), bad
    f = pqgpu.File(data)
    b = pqgpu.Batch(gpu_ctx)
    ids = {(rg, col): b.add_file_chunk(f, rg, col)[0] for rg in range(f.num_row_groups) for col in range(f.num_columns)}
    for rounds in (3, 1, 1, 2, 1):
        for _ in range(rounds):
            b.decode()
        e = b.sync()
        assert (e is None) == (not bad), e
        for rg, col, r in orc:
            g = b.status(ids[(rg, col)])
            where = f"{which} x{rounds} rg{rg} col{col}"
            if isinstance(r, O.OracleError):
                assert g is not None and (g.code, g.page) == (r.code, r.page), (where, g, r)
            else:
                assert g is None, (where, g)
                pqtest.assert_chunk_equal(b.result(ids[(rg, col)]), r, where)
    b.close()


def _flip_def(name, col, to_null, page=1):
    """Fixture `name` with one definition level of column `col`'s data page `page` changed inside a
    bit-packed run (else the value of its first RLE run that has one): max_def -> max_def - 1
    (non-null values become null) or back (nulls become non-null). The value bytes stay as they were."""
    import io
    import os
    import sys
    import pyarrow.parquet as pq
    sys.path.insert(0, os.path.join(os.path.dirname(pqtest.GOLDEN), "..", "tools"))
    import pqinspect
    buf = bytearray(pqtest.load(name))
    sc = pq.ParquetFile(io.BytesIO(bytes(buf))).metadata.schema.column(col)
    mr, md = sc.max_repetition_level, sc.max_definition_level
    ph, j = [(ph, j) for ph, j in pqinspect.pages(bytes(buf), 0, col) if ph[1] == 0][page]
    assert ph[5][2] == 0  # PLAIN values
    p = j
    if mr:
        p += 4 + int.from_bytes(buf[p:p + 4], "little")
    end = p + 4 + int.from_bytes(buf[p:p + 4], "little")
    p += 4
    bw = md.bit_length()
    src, dst = (md, md - 1) if to_null else (md - 1, md)
    rle = None
    while p < end:
        h, q = pqinspect.uvar(buf, p)
        if h & 1:
            n = (h >> 1) * 8
            for k in range(n):
                bit = (q * 8) + k * bw
                v = (int.from_bytes(buf[bit // 8:bit // 8 + 2], "little") >> (bit % 8)) & ((1 << bw) - 1)
                if v == src:
                    x = int.from_bytes(buf[bit // 8:bit // 8 + 2], "little")
                    x = (x & ~(((1 << bw) - 1) << (bit % 8))) | (dst << (bit % 8))
                    buf[bit // 8:bit // 8 + 2] = x.to_bytes(2, "little")
                    return bytes(buf)
            p = q + (h >> 1) * bw
        else:
            if rle is None and buf[q] == src:
                rle = q
            p = q + (bw + 7) // 8
    assert rle is not None, "no level to flip"
    buf[rle] = dst  # no bit-packed run holds one: a whole RLE run changes
    return bytes(buf)


@pytest.mark.parametrize("to_null", [True, False])
@pytest.mark.parametrize("name,col", [("edge_nulls_v1", 0), ("types_v1", 1), ("types_v1", 5), ("cfg4_small", 0), ("cfg4_small", 2)])
def test_copies_early_count_miss(gpu_ctx, name, col, to_null):
    """Serial batches start their PLAIN copies on non-null counts speculated from the pages' value
    bytes (host.cpp copies_early). A page whose definition levels hold one null more than its value
    bytes imply (the reference reads one value less and ignores the last one) or one null less (it
    runs out of values: io.EOF on that page) misses the speculation; the batch is decoded again in
    the serial order and every chunk equals the oracle, errors at the reference's (code, page)."""
    data = _flip_def(name, col, to_null)
    orc = pqtest.oracle_decode(data)
    gpu = _gpu_decode(gpu_ctx, data)
    for rg, c, r in orc:
        g = gpu[(rg, c)]
        where = f"{name} col{col} to_null={to_null}: rg{rg} col{c}"
        if isinstance(r, O.OracleError):
            assert isinstance(g, pqgpu.DecodeError), f"{where}: oracle error {r} but GPU decoded"
            assert (g.code, g.page) == (r.code, r.page), f"{where}: {g} vs {r}"
        else:
            assert not isinstance(g, pqgpu.DecodeError), f"{where}: GPU error {g}"
            pqtest.assert_chunk_equal(g, r, where)
