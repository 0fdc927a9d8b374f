"""The streaming row-group pipeline (pqgpu_pipeline_*: FileReader.readRowGroupData called row
group after row group, chunk_reader.go:375-404, file_reader.go:187-198) and partial chunk results
(the pages before a failing page, data_store.go:236-260). Every chunk a pipeline returns must equal
the oracle, whatever the depth / thread count; a page-level failure keeps the decoded prefix."""
import ctypes
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import rawpq  # noqa: E402

import pqgpu  # noqa: E402
import pqtest  # noqa: E402
import py_oracle as O  # noqa: E402

PAGE_ROWS = [3000, 5000, 4000, 2000]
BAD = {"i": 2, "s": 1}  # column -> data page whose dictionary index is out of range


def bad_page_file(seed=0):
    """i: INT32 OPTIONAL dictionary (100 entries, 7-bit indices), s: BYTE_ARRAY OPTIONAL dictionary
    (50 entries), d: DOUBLE REQUIRED PLAIN. Page BAD[col] of i / s holds index 105 / 55 at its
    value 17 (type_dict.go:52-54 fails that page). Returns (file, expected per column: values and
    def levels of every row)."""
    rng = np.random.default_rng(900 + seed)
    n = sum(PAGE_ROWS)
    d32 = rng.integers(-2**31, 2**31 - 1, 100, dtype=np.int64).astype(np.int32)
    vocab = sorted({bytes(rng.integers(97, 123, int(rng.integers(1, 12)), dtype=np.uint8)) for _ in range(200)})[:50]
    cols = {"i": (rng.integers(0, 100, n), rng.random(n) < 0.2, 100), "s": (rng.integers(0, 50, n), rng.random(n) < 0.1, 50),
            "d": (rng.random(n), np.zeros(n, bool), 0)}
    chunks, expect = [], {}
    for name, (vals, nulls, dsz) in cols.items():
        dl = (~nulls).astype(int).tolist()
        pages = []
        if name == "i":
            pages.append(rawpq.dict_page_ref("INT32", d32))
        if name == "s":
            pages.append(rawpq.dict_page_ref("BYTE_ARRAY", vocab))
        at = 0
        for k, pr in enumerate(PAGE_ROWS):
            sl = slice(at, at + pr)
            at += pr
            nn = [int(x) for x in vals[sl][~nulls[sl]]]
            if name == "d":
                pages.append(rawpq.data_page_v1_ref(pr, "PLAIN", rawpq.plain_encode("DOUBLE", vals[sl]), None, 0))
                continue
            if BAD[name] == k:
                nn[17] = dsz + 5  # still fits the bits.Len(len(dict)) index width
            pages.append(rawpq.data_page_v1_ref(pr, "RLE_DICTIONARY", rawpq.dict_values_section(nn, dsz), dl[sl], 1))
        expect[name] = (vals, nulls)
        chunks.append((pages, n, name != "d"))
    schema = [[(4, rawpq.BIN, "schema"), (5, rawpq.I32, 3)], rawpq.schema_leaf("i", "INT32", "OPTIONAL"),
              rawpq.schema_leaf("s", "BYTE_ARRAY", "OPTIONAL"), rawpq.schema_leaf("d", "DOUBLE", "REQUIRED")]
    leaves = [("i", "INT32"), ("s", "BYTE_ARRAY"), ("d", "DOUBLE")]
    return rawpq.write_file_schema(schema, leaves, [(n, chunks)]), (d32, vocab, expect)


def test_oracle_bad_pages():
    data, _ = bad_page_file()
    f = O.File(data)
    for c, name in enumerate(["i", "s"]):
        with pytest.raises(O.OracleError) as ei:
            f.read_chunk(0, c)
        assert (ei.value.code, ei.value.page) == (5, BAD[name])
    f.read_chunk(0, 2)


@pytest.mark.gpu
def test_gpu_partial_results(gpu_ctx):
    data, (d32, vocab, expect) = bad_page_file()
    f = pqgpu.File(data)
    b = pqgpu.Batch(gpu_ctx)
    ids = [b.add_file_chunk(f, 0, c)[0] for c in range(3)]
    b.decode()
    b.sync()
    for c, name in enumerate(["i", "s"]):
        part, e = b.result(ids[c], partial=True)
        assert e is not None and (e.code, e.page) == (5, BAD[name])
        slots = sum(PAGE_ROWS[:BAD[name]])
        vals, nulls = expect[name]
        keep = ~nulls[:slots]
        assert part.num_slots == slots and part.num_values == int(keep.sum())
        np.testing.assert_array_equal(part.validity_bits()[:slots].astype(bool), keep)
        idx = vals[:slots][keep]
        if name == "i":
            np.testing.assert_array_equal(part.values, d32[idx])
        else:
            want = [vocab[k] for k in idx]
            got = [part.payload[part.offsets[k]:part.offsets[k + 1]] for k in range(len(want))]
            assert got == want
        with pytest.raises(pqgpu.DecodeError):
            b.result(ids[c])
    r = b.result(ids[2])
    np.testing.assert_array_equal(r.values, expect["d"][0].view(np.uint64))  # raw bits (Q11)
    b.close()


def _files_for_pipeline():
    return [n for n in ("cfg2_v2_small", "cfg5_small", "cfg4_small", "types_v2", "cfg3_small", "edge_nulls_v1")
            if n in pqtest.ALL]


@pytest.mark.gpu
@pytest.mark.parametrize("depth,threads,device_index", [(1, 1, False), (2, 2, False), (4, 3, False), (2, 2, True),
                                                        (3, 3, True)])
@pytest.mark.parametrize("name", _files_for_pipeline())
def test_gpu_pipeline_parity(gpu_ctx, name, depth, threads, device_index):
    """device_index: each row group's byte range is made resident and its page headers walked on the
    GPU (pagewalk.hip); the results must not change."""
    data = pqtest.load(name)
    orc = {(rg, col): r for rg, col, r in pqtest.oracle_decode(data)}
    f = pqgpu.File(data)
    p = pqgpu.Pipeline(gpu_ctx, f, depth=depth, threads=threads, device_index=device_index)
    seen = []
    for rg, b, err in p:
        seen.append(rg)
        for col in range(f.num_columns):
            want = orc[(rg, col)]
            e = b.status(col)
            if isinstance(want, O.OracleError):
                assert e is not None and (e.code, e.page) == (want.code, want.page), (name, rg, col)
            else:
                assert e is None, (name, rg, col, e)
                pqtest.assert_chunk_equal(b.result(col), want, f"{name} rg{rg} col{col}")
    assert seen == list(range(f.num_row_groups))
    st = p.stats()
    assert st["row_groups"] == f.num_row_groups and st["chunks"] == f.num_row_groups * f.num_columns
    assert (st["index_ms"] > 0) == device_index
    # every device walk reported on the first read-back
    assert st["ix_polls"] == 0 and st["ix_unreported"] == 0, st
    p.close()


@pytest.mark.gpu
def test_gpu_pipeline_subset_and_errors(gpu_ctx):
    data, _ = bad_page_file()
    f = pqgpu.File(data)
    p = pqgpu.Pipeline(gpu_ctx, f, row_groups=[0, 0], cols=[2, 0], depth=2)
    out = list((rg, b.status(0), b.status(1)) for rg, b, _ in p)
    assert len(out) == 2
    for rg, e_d, e_i in out:
        assert rg == 0 and e_d is None and e_i is not None and (e_i.code, e_i.page) == (5, 2)
    p.close()


@pytest.mark.gpu
def test_gpu_pipeline_release_protocol(gpu_ctx):
    """Asking for row group k + depth while row group k is still held is an argument error, not a hang."""
    data = pqtest.load(_files_for_pipeline()[0])
    f = pqgpu.File(data)
    if f.num_row_groups < 2:
        pytest.skip("needs two row groups")
    L = pqgpu.lib()
    h = ctypes.c_void_p()
    err = pqgpu.Error()
    opts = pqgpu.PipelineOpts(1, 1, 0, 0)
    assert L.pqgpu_pipeline_create(gpu_ctx._h, f._h, None, 0, None, 0, ctypes.byref(opts), ctypes.byref(h),
                                   ctypes.byref(err)) == 0
    b, rg = ctypes.c_void_p(), ctypes.c_int32()
    L.pqgpu_pipeline_next(h, ctypes.byref(b), ctypes.byref(rg), ctypes.byref(err))
    assert b.value and rg.value == 0
    b2 = ctypes.c_void_p()
    assert L.pqgpu_pipeline_next(h, ctypes.byref(b2), ctypes.byref(rg), ctypes.byref(err)) == 11  # PQ_ERR_ARG
    assert L.pqgpu_pipeline_release(h, b) == 0
    assert L.pqgpu_pipeline_next(h, ctypes.byref(b2), ctypes.byref(rg), ctypes.byref(err)) in (0, 5, 1, 2, 3)
    assert b2.value and rg.value == 1
    L.pqgpu_pipeline_destroy(h)


@pytest.mark.gpu
def test_gpu_pipeline_cfg5_replica(gpu_ctx):
    """cfg5's generator: pyarrow row-group templates replicated behind a rewritten footer
    (SNAPPY V1, 64 columns) — every chunk through the pipeline equals the oracle."""
    import workloads as W
    data, _ = W.gen_cfg5(rows=3 * 20000, rg_rows=20000)
    orc = {(rg, col): r for rg, col, r in pqtest.oracle_decode(data)}
    f = pqgpu.File(data)
    p = pqgpu.Pipeline(gpu_ctx, f, depth=2, threads=2, device_index=True)
    n = 0
    for rg, b, err in p:
        assert err is None
        for col in range(f.num_columns):
            pqtest.assert_chunk_equal(b.result(col), orc[(rg, col)], f"cfg5 rg{rg} col{col}")
        n += 1
    assert n == 3
    p.close()


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["crc_v1", "crc_v1_flipped"])
def test_gpu_pipeline_device_index_crc(gpu_ctx, name):
    """WithCRC32Validation through the device-index pipeline (checksums on the GPU): every chunk's
    outcome equals the host-walk pipeline's (the flipped byte fails its page with PQ_ERR_CRC)."""
    data = pqtest.load(name)
    f = pqgpu.File(data)
    out = {}
    for dix in (False, True):
        p = pqgpu.Pipeline(gpu_ctx, f, depth=2, threads=2, validate_crc=True, device_index=dix)
        for rg, b, _err in p:  # (an assertion below leaves p to pqgpu's exit-time cleanup)
            for col in range(f.num_columns):
                e = b.status(col)
                if e is not None:
                    got = (e.code, e.page)
                else:
                    r = b.result(col)
                    got = (r.num_slots, r.num_values, r.dLevels.tobytes(),
                           r.payload if r.offsets is not None else np.asarray(r.values_raw).tobytes())
                out.setdefault((rg, col), []).append(got)
        p.close()
    for k, (host, dev) in out.items():
        assert host == dev, (name, k)
    if name == "crc_v1_flipped":
        assert any(isinstance(v[0], tuple) and v[0][0] == pqgpu.PQ_ERR_CRC for v in out.values())
