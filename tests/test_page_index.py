"""On-device page index (parquet-go-1_amd/csrc/pagewalk.hip): readPages'
page-header loop (chunk_reader.go:182-263), the Thrift decode of every PageHeader (readThrift
helpers.go:103-109) and readPageBlock's CRC32 check (chunk_reader.go:173-177) run on the GPU over
file bytes resident in HBM.

Parity, in three layers:
- every header the device walk decoded equals the host's decode of the same bytes (pqgpu_parse_page_header,
  the parser the plain path and the oracle cross-checks use), at the same file offsets, in the same
  chain order (the Python walk below restates readPages' loop);
- a chunk the walk did not take (IX_FALLBACK) is one the host path rejects, or one whose bytes are
  not all resident;
- decoding through indexed chunks gives exactly the oracle's result: values, levels, the same error
  class on the same page (CRC32 failures included) — on every fixture, the reference's
  must-not-crash images, and seeded header corruptions.
"""
import os
import sys

import numpy as np
import pytest

import pqgpu
import pqtest
import py_oracle as O

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))

pytestmark = pytest.mark.gpu


def _host_chain(data, m):
    """readPages' header loop restated (chunk_reader.go:182-263): [(offset, PageHeader)] until
    TotalCompressedSize is consumed, or None where the host stops with an error in the chain."""
    off = m.dictionary_page_offset if m.dictionary_page_offset >= 0 else m.data_page_offset
    count, out = 0, []
    while m.total_compressed_size - count > 0:
        if off < 0 or off >= len(data):
            return None
        h, n = pqgpu.parse_page_header(data[off:])
        if h is None:
            return None
        out.append((off, h))
        off += n
        count += n
        if h.compressed_page_size < 0 or h.uncompressed_page_size < 0 or off + h.compressed_page_size > len(data):
            return None
        off += h.compressed_page_size
        count += h.compressed_page_size
        if h.type == 2 and m.dictionary_page_offset >= 0 and m.dictionary_page_offset != off:
            if m.data_page_offset < 0:
                return None
            count += m.data_page_offset - off
            off = m.data_page_offset
    return out


def _all_chunks(f):
    return [(rg, c) for rg in range(f.num_row_groups) for c in range(f.num_columns)]


def _decode_indexed(ctx, data, validate_crc=False, per_row_group=False):
    """{(rg, col): ColumnData | DecodeError} through indexed chunks, and the indexes built."""
    f = pqgpu.File(data)
    chunks, plain = [], []  # chunks whose metadata is unreadable take the plain path (its error)
    for rg, c in _all_chunks(f):
        try:
            f.chunk_meta(rg, c)
            chunks.append((rg, c))
        except pqgpu.DecodeError:
            plain.append((rg, c))
    if per_row_group:
        ixs, where = [], {}
        for rg in range(f.num_row_groups):
            mine = [k for k in chunks if k[0] == rg]
            ix = pqgpu.PageIndex.for_chunks(ctx, f, mine, validate_crc)
            ixs.append((ix, rg))
            where.update({k: (ix, i) for i, k in enumerate(mine)})
    else:
        ix = pqgpu.PageIndex.for_chunks(ctx, f, chunks, validate_crc, whole_file=True)
        ixs = [(ix, None)]
        where = {k: (ix, i) for i, k in enumerate(chunks)}
    b = pqgpu.Batch(ctx)
    ids = {}
    for rg, c in _all_chunks(f):
        if (rg, c) in where:
            ix, k = where[(rg, c)]
            cid, _e = b.add_indexed_chunk(ix, k, f, c, validate_crc)
        else:
            cid, _e = b.add_file_chunk(f, rg, c, validate_crc)
        ids[(rg, c)] = cid
    b.upload()
    for ix, _ in ixs:
        ix.close()  # the resident bytes are no longer needed once the upload has gathered them
    b.decode()
    b.sync()
    out = {}
    for k, cid in ids.items():
        e = b.status(cid)
        out[k] = e if e is not None else b.result(cid)
    b.close()
    return out


def _check_against_oracle(name, data, got):
    orc = pqtest.oracle_decode(data)
    for rg, col, r in orc:
        g = got[(rg, col)]
        where = f"{name} rg{rg} col{col}"
        if isinstance(r, O.OracleError):
            assert isinstance(g, pqgpu.DecodeError), f"{where}: oracle error {r} but decoded"
            assert (g.code, g.page) == (r.code, r.page), f"{where}: {g} vs {r}"
        else:
            assert not isinstance(g, pqgpu.DecodeError), f"{where}: error {g}"
            pqtest.assert_chunk_equal(g, r, where)


def _oracle_ok(data):
    try:
        O.File(data)
        return True
    except O.OracleError:
        return False


@pytest.mark.parametrize("name", pqtest.ALL)
def test_headers_match_host_walk(gpu_ctx, name):
    data = pqtest.load(name)
    if not _oracle_ok(data):
        pytest.skip("footer-level error")
    f = pqgpu.File(data)
    chunks = _all_chunks(f)
    ix = pqgpu.PageIndex.for_chunks(gpu_ctx, f, chunks, whole_file=True)  # fixtures: readable metadata
    pb = pqgpu.Batch(None)  # plan-only: the host path's verdict on each chunk
    for k, (rg, c) in enumerate(chunks):
        n, st = ix.chunk(k)
        host = _host_chain(data, f.chunk_meta(rg, c))
        if st == pqgpu.IX_OK:
            assert host is not None, f"{name} rg{rg} c{c}: device walked a chain the host stops in"
            assert n == len(host), (name, rg, c, n, len(host))
            for i, (off, h) in enumerate(host):
                d = ix.page(k, i)
                assert d.header_offset == off, (name, rg, c, i)
                assert d.key() == h.key(), (name, rg, c, i, d.key(), h.key())
        else:
            _cid, e = pb.add_file_chunk(f, rg, c)
            assert host is None or e is not None, f"{name} rg{rg} c{c}: fallback on a chunk the host accepts"
    ix.close()
    pb.close()


@pytest.mark.parametrize("name", pqtest.ALL)
def test_indexed_decode_parity(gpu_ctx, name):
    data = pqtest.load(name)
    if not _oracle_ok(data):
        pytest.skip("footer-level error")
    _check_against_oracle(name, data, _decode_indexed(gpu_ctx, data))


@pytest.mark.parametrize("name", ["cfg2_v2_small", "cfg4_small", "types_v2", "cfg3_dict64k", "edge_tiny_pages"])
def test_indexed_row_group_ranges(gpu_ctx, name):
    """One resident byte range per row group (the pipeline's use): same results as the oracle."""
    data = pqtest.load(name)
    _check_against_oracle(name, data, _decode_indexed(gpu_ctx, data, per_row_group=True))


def test_tiny_pages_take_the_device_walk(gpu_ctx):
    """edge_tiny_pages: many small pages per chunk, all walked on the device (no fallback)."""
    data = pqtest.load("edge_tiny_pages")
    f = pqgpu.File(data)
    chunks = _all_chunks(f)
    ix = pqgpu.PageIndex.for_chunks(gpu_ctx, f, chunks, whole_file=True)
    pages = [ix.chunk(k) for k in range(len(chunks))]
    assert all(st == pqgpu.IX_OK for _n, st in pages)
    assert sum(n for n, _ in pages) >= 64 * len(chunks) // 4  # several table flushes per chunk
    ix.close()


@pytest.mark.parametrize("name", ["crc_v1", "crc_v1_flipped"])
def test_crc_on_device(gpu_ctx, name):
    """WithCRC32Validation: the device checksums decide, with the reference's error class and page."""
    import zlib
    data = pqtest.load(name)
    f = pqgpu.File(data)
    chunks = _all_chunks(f)
    ix = pqgpu.PageIndex.for_chunks(gpu_ctx, f, chunks, validate_crc=True, whole_file=True)
    checked = 0
    for k, (rg, c) in enumerate(chunks):
        n, st = ix.chunk(k)
        assert st == pqgpu.IX_OK
        for i in range(n):
            h = ix.page(k, i)
            if not h.flags & pqgpu.PH_CRC:
                continue
            body = data[h.header_offset + h.header_len: h.header_offset + h.header_len + h.compressed_page_size]
            assert h.flags & pqgpu.PH_CRC_CHECKED
            assert bool(h.flags & pqgpu.PH_CRC_OK) == (zlib.crc32(body) == (h.crc & 0xffffffff)), (k, i)
            checked += 1
    assert checked > 0
    ix.close()
    got = _decode_indexed(gpu_ctx, data, validate_crc=True)
    plain = pqgpu.Batch(gpu_ctx)
    for (rg, c), g in sorted(got.items()):
        _cid, e = plain.add_file_chunk(f, rg, c, validate_crc=True)
        if e is not None:
            assert isinstance(g, pqgpu.DecodeError) and (g.code, g.page, g.msg) == (e.code, e.page, e.msg)
    plain.close()
    if name == "crc_v1_flipped":
        assert any(isinstance(g, pqgpu.DecodeError) and g.code == pqgpu.PQ_ERR_CRC for g in got.values())


def test_crc_sizes(gpu_ctx):
    """CRC32 of blocks of every size class (empty, sub-segment, unaligned, multi-segment) against zlib:
    a synthetic chunk of V1 pages whose bodies are random bytes, indexed and checked on the device."""
    import zlib
    import rawpq
    rng = np.random.default_rng(11)
    sizes = [0, 1, 3, 4, 5, 255, 256, 257, 1023, 1024, 4097, 65536 + 7, 300001]
    pages = []
    for s in sizes:
        body = rng.integers(0, 256, s, dtype=np.uint8).tobytes()
        good = s % 2 == 0
        pages.append((body, zlib.crc32(body) if good else zlib.crc32(body) ^ 1))
    blob, metas = rawpq.crc_probe_chunk(pages)
    buf = pqgpu.DeviceBuffer(gpu_ctx, blob)
    ix = pqgpu.PageIndex(gpu_ctx, buf.ptr.value, 0, len(blob), metas, validate_crc=True, keep=buf)
    n, st = ix.chunk(0)
    assert st == pqgpu.IX_OK and n == len(sizes)
    for i, s in enumerate(sizes):
        h = ix.page(0, i)
        assert h.compressed_page_size == s
        assert h.flags & pqgpu.PH_CRC_CHECKED
        assert bool(h.flags & pqgpu.PH_CRC_OK) == (s % 2 == 0), (i, s)
    ix.close()


def test_partial_residency_falls_back(gpu_ctx):
    """Bytes cut short of a chunk: the walk hands that chunk to the host, results unchanged."""
    data = pqtest.load("cfg2_v2_small")
    f = pqgpu.File(data)
    chunks = _all_chunks(f)
    m = f.chunk_meta(*chunks[-1])
    st0 = m.dictionary_page_offset if m.dictionary_page_offset >= 0 else m.data_page_offset
    cut = st0 + m.total_compressed_size // 2  # the last chunk is only half resident
    buf = pqgpu.DeviceBuffer(gpu_ctx, data[:cut])
    metas = [f.chunk_meta(rg, c) for rg, c in chunks]
    ix = pqgpu.PageIndex(gpu_ctx, buf.ptr.value, 0, cut, metas, keep=buf)
    assert ix.chunk(len(chunks) - 1)[1] == pqgpu.IX_FALLBACK
    assert ix.chunk(0)[1] == pqgpu.IX_OK
    b = pqgpu.Batch(gpu_ctx)
    ids = []
    for k, (rg, c) in enumerate(chunks):
        cid, e = b.add_indexed_chunk(ix, k, f, c)
        assert e is None
        ids.append(cid)
    b.upload()
    ix.close()
    b.decode()
    assert b.sync() is None
    orc = pqtest.oracle_decode(data)
    for (rg, c, r), cid in zip(orc, ids):
        pqtest.assert_chunk_equal(b.result(cid), r, f"rg{rg} c{c}")
    b.close()


@pytest.mark.parametrize("name", ["cfg5_small", "cfg2_snappy_v1", "dba_v1_snappy"])
def test_indexed_snappy_decoded_twice_after_release(gpu_ctx, name):
    """SNAPPY blocks of indexed chunks are gathered from the resident bytes at upload; the index and
    its device buffer are released before the first decode, and a second decode of the same batch
    (the bench's pattern) still equals the oracle."""
    data = pqtest.load(name)
    f = pqgpu.File(data)
    chunks = _all_chunks(f)
    ix = pqgpu.PageIndex.for_chunks(gpu_ctx, f, chunks, whole_file=True)
    b = pqgpu.Batch(gpu_ctx)
    ids = []
    for k, (rg, c) in enumerate(chunks):
        cid, e = b.add_indexed_chunk(ix, k, f, c)
        ids.append(cid)
    b.upload()
    ix.close()
    orc = pqtest.oracle_decode(data)
    for rep in range(2):
        b.decode()
        b.sync()
        for (rg, c, r), cid in zip(orc, ids):
            if isinstance(r, O.OracleError):
                continue
            pqtest.assert_chunk_equal(b.result(cid), r, f"{name} pass {rep} rg{rg} c{c}")
    b.close()


def test_must_not_crash_indexed(gpu_ctx):
    """The reference's fuzz regression images through the indexed path: the oracle's outcome."""
    d = os.path.join(pqtest.GOLDEN, "must_not_crash")
    n = 0
    for fn in sorted(os.listdir(d)):
        data = open(os.path.join(d, fn), "rb").read()
        if not _oracle_ok(data):
            continue
        _check_against_oracle(fn, data, _decode_indexed(gpu_ctx, data))
        n += 1
    assert n > 0


@pytest.mark.parametrize("seed", range(6))
def test_corrupted_headers(gpu_ctx, seed):
    """Seeded corruptions of page-header bytes: the indexed path returns the oracle's outcome
    (whichever of device walk or host fallback decides it)."""
    rng = np.random.default_rng(100 + seed)
    base = pqtest.load(["types_v1", "types_v2", "cfg4_small", "types_dict", "edge_nulls_v1", "cfg3_small"][seed])
    f = pqgpu.File(base)
    hdrs = []
    for rg, c in _all_chunks(f):
        for off, h in _host_chain(base, f.chunk_meta(rg, c)) or []:
            hdrs.append((off, h.header_len))
    for trial in range(8):
        data = bytearray(base)
        for _ in range(int(rng.integers(1, 4))):
            off, hl = hdrs[int(rng.integers(len(hdrs)))]
            p = off + int(rng.integers(hl))
            data[p] = int(rng.integers(256))
        data = bytes(data)
        if not _oracle_ok(data):
            continue
        _check_against_oracle(f"seed{seed}.{trial}", data, _decode_indexed(gpu_ctx, data))


@pytest.mark.parametrize("no_grow", [False, True])
def test_table_overflow(gpu_ctx, monkeypatch, no_grow):
    """A header table too small for the walk (PQ_IX_CAP forces the first capacity): the CRC pass
    checksums nothing of an overflowed table, the build is rerun larger, or — when it may not grow
    (PQ_IX_NOGROW) — keeps no entries and hands every chunk to the host walk. Results equal the
    oracle's either way, with CRC validation on."""
    data = pqtest.load("edge_tiny_pages")
    f = pqgpu.File(data)
    chunks = _all_chunks(f)
    monkeypatch.setenv("PQ_IX_CAP", "8")
    if no_grow:
        monkeypatch.setenv("PQ_IX_NOGROW", "1")
    ix = pqgpu.PageIndex.for_chunks(gpu_ctx, f, chunks, validate_crc=True, whole_file=True)
    st = ix.stats()
    assert st["polls"] == 0 and st["unreported"] == 0, st
    if no_grow:
        assert st["overflowed"] == 1 and st["fallback_chunks"] == len(chunks), st
        assert all(ix.chunk(k) == (0, pqgpu.IX_FALLBACK) for k in range(len(chunks)))
    else:
        assert st["overflowed"] == 0 and st["fallback_chunks"] == 0, st
    ix.close()
    _check_against_oracle("edge_tiny_pages", data, _decode_indexed(gpu_ctx, data, validate_crc=True))


@pytest.mark.parametrize("name", ["cfg2_v2_small", "cfg5_small", "edge_tiny_pages"])
def test_build_stats_clean(gpu_ctx, name):
    """Every chunk's completion marker (a per-build generation) is visible at the first read-back:
    no polls, no unreported chunk, across repeated builds that reuse the same scratch."""
    data = pqtest.load(name)
    f = pqgpu.File(data)
    for _ in range(3):
        ix = pqgpu.PageIndex.for_chunks(gpu_ctx, f, _all_chunks(f), whole_file=True)
        st = ix.stats()
        ix.close()
        assert st == {"polls": 0, "unreported": 0, "fallback_chunks": 0, "overflowed": 0, "stale_entries": 0}, (name, st)


def _stale_entries_body(gpu_ctx, name):
    """(run in a diagnostic-library process: PQ_IX_TEST_SKIP_STORE exists only in that build)"""
    data = pqtest.load(name)
    f = pqgpu.File(data)
    chunks = _all_chunks(f)
    k = len(chunks) - 1  # the chunk whose stores are dropped
    mine = [chunks[k]]
    os.environ.pop("PQ_IX_TEST_SKIP_STORE", None)
    ix = pqgpu.PageIndex.for_chunks(gpu_ctx, f, mine, whole_file=True)  # fills the scratch table
    pages, status = ix.chunk(0)
    assert status == pqgpu.IX_OK and pages > 0
    ix.close()
    os.environ["PQ_IX_TEST_SKIP_STORE"] = "0"
    ix = pqgpu.PageIndex.for_chunks(gpu_ctx, f, mine, whole_file=True)
    st = ix.stats()
    assert ix.chunk(0) == (0, pqgpu.IX_FALLBACK), (name, st)
    assert st["stale_entries"] == pages and st["fallback_chunks"] == 1 and st["unreported"] == 0, (name, st)
    ix.close()
    # the whole file with one chunk's stores dropped: that chunk is walked by the host, the others
    # by the device, and every result equals the oracle's
    os.environ["PQ_IX_TEST_SKIP_STORE"] = str(k)
    ix = pqgpu.PageIndex.for_chunks(gpu_ctx, f, chunks, whole_file=True)
    st = ix.stats()
    assert st["fallback_chunks"] == 1 and st["stale_entries"] >= 0, st
    assert ix.chunk(k)[1] == pqgpu.IX_FALLBACK and all(ix.chunk(j)[1] == pqgpu.IX_OK for j in range(k))
    ix.close()
    got = _decode_indexed(gpu_ctx, data)
    os.environ.pop("PQ_IX_TEST_SKIP_STORE", None)
    _check_against_oracle(name, data, got)


STALE_SCRIPT = """
import sys
sys.path[:0] = sys.argv[2:5]
import pqgpu, test_page_index as T
T._stale_entries_body(pqgpu.Context(0), sys.argv[1])
print("STALE-OK")
"""


@pytest.mark.parametrize("name", ["edge_tiny_pages", "cfg2_v2_small"])
def test_stale_entries_dropped(name):
    """Table entries carry the build's generation stamp. A chunk whose walk reports success with the
    right page count but whose table stores never landed (PQ_IX_TEST_SKIP_STORE, a hook of the
    diagnostic library only: its slots are reserved and left as they were — here holding the
    previous build's entries for the same chunk, same slots, same count) must not be trusted: its
    entries are dropped as stale, the count no longer adds up, the chunk falls back to the host
    walk, and the decode still equals the oracle."""
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    diag = os.path.join(root, "parquet-go-1_amd", "lib", "libpqgpu_diag.so")
    assert os.path.exists(diag), "make -C parquet-go-1_amd diag"
    env = dict(os.environ, PQGPU_LIB=diag)
    env.pop("PQ_IX_TEST_SKIP_STORE", None)
    tests = os.path.dirname(os.path.abspath(__file__))
    r = subprocess.run([sys.executable, "-c", STALE_SCRIPT, name, tests, os.path.join(root, "parquet-go-1_amd"),
                        os.path.join(root, "oracle")], env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0 and "STALE-OK" in r.stdout, r.stdout[-2000:] + r.stderr[-2000:]


def test_skip_store_hook_absent_from_product(gpu_ctx, monkeypatch):
    """The production library ignores PQ_IX_TEST_SKIP_STORE: every chunk is walked on the device."""
    data = pqtest.load("edge_tiny_pages")
    f = pqgpu.File(data)
    chunks = _all_chunks(f)
    monkeypatch.setenv("PQ_IX_TEST_SKIP_STORE", "0")
    ix = pqgpu.PageIndex.for_chunks(gpu_ctx, f, chunks, whole_file=True)
    st = ix.stats()
    assert st["fallback_chunks"] == 0 and st["stale_entries"] == 0, st
    ix.close()
