"""Dictionary tiles of 4-byte values decoded in groups (k_values_dict2, kernels.hip do_dict2;
host.cpp groups a page's consecutive 4,096-value tiles when a batch has many): index streams of bit
widths 1, 8 and 10 that mix RLE runs with bit-packed runs (hybrid_decoder.go:142-165), runs that
straddle tile boundaries, REQUIRED and OPTIONAL columns, a page whose last group has one tile, and
an out-of-range index in the second tile of a group (type_dict.go:52-54). Grouped decoding must
give the oracle's values, and its error at the same page."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import rawpq  # noqa: E402

import pqtest  # noqa: E402
import py_oracle as O  # noqa: E402

PAGE_VALUES = [20000, 4096 * 3 + 5, 9000]
COLS = {"bw1": 2, "bw8": 200, "bw10": 700}  # dictionary entries


def hybrid_mixed(rng, idx, bw):
    """RLE/bit-packed hybrid stream of idx: alternating bit-packed runs (multiples of 8 values) and
    RLE runs of repeated indices (the caller repeats them in idx)."""
    out = b""
    i, n = 0, len(idx)
    while i < n:
        j = i
        while j < n and idx[j] == idx[i]:
            j += 1
        if j - i >= 16:  # a repeat: one RLE run
            out += rawpq.uvar((j - i) << 1) + int(idx[i]).to_bytes((bw + 7) // 8, "little")
            i = j
            continue
        k = min(n, i + 8 * int(rng.integers(1, 64)))  # a bit-packed run of 8 g values (the last one padded)
        g = (k - i + 7) // 8
        vals = list(idx[i:k]) + [0] * (g * 8 - (k - i))
        out += rawpq.uvar((g << 1) | 1) + rawpq.bitpack(vals, bw)
        i = k
    return bytes([bw]) + out


def build(seed, bad=False, optional=False):
    rng = np.random.default_rng(900 + seed)
    names = list(COLS)
    chunks = []
    expect = {}
    for name in names:
        k = COLS[name]
        bw = int(k).bit_length() if k > 2 else 1
        vocab = [int(x) for x in rng.integers(-2**31, 2**31 - 1, k)]
        pages = [rawpq.dict_page_ref("INT32", vocab)]
        vals, dls = [], []
        for p, nv in enumerate(PAGE_VALUES):
            nulls = rng.random(nv) < (0.1 if optional else 0.0)
            dl = (~nulls).astype(int)
            nn = int(dl.sum())
            idx = rng.integers(0, k, nn)
            at = 0
            while at < nn:  # repeats (RLE runs), some across the 4,096-value tile boundaries
                ln = int(rng.integers(16, 3000))
                idx[at:at + ln] = idx[at]
                at += ln + int(rng.integers(100, 5000))
            if bad and name == "bw10" and p == 1:
                idx[4096 + 77] = k + 3  # in the second tile of the page's first group; fits 10 bits
            body = hybrid_mixed(rng, idx, bw)
            pages.append(rawpq.data_page_v1_ref(nv, "RLE_DICTIONARY", body, dl.tolist() if optional else None,
                                                1 if optional else 0))
            vals += [vocab[i] if i < k else None for i in idx]
            dls.append(dl)
        chunks.append((pages, sum(PAGE_VALUES), True))
        expect[name] = vals
    schema = [[(4, rawpq.BIN, "schema"), (5, rawpq.I32, len(names))]]
    schema += [rawpq.schema_leaf(name, "INT32", "OPTIONAL" if optional else "REQUIRED") for name in names]
    leaves = [(name, "INT32") for name in names]
    return rawpq.write_file_schema(schema, leaves, [(sum(PAGE_VALUES), chunks)]), expect


@pytest.mark.parametrize("optional", [False, True])
def test_oracle_dict_groups(optional):
    data, expect = build(0, optional=optional)
    f = O.File(data)
    for c, name in enumerate(COLS):
        r = f.read_chunk(0, c)
        np.testing.assert_array_equal(np.asarray(pqtest.oracle_values(r)), np.asarray(expect[name], np.int32), err_msg=name)


def build_bw0(seed, optional=False, entries=1):
    """INT32 RLE_DICTIONARY pages of index bit width 0 (parquet-mr sizes the width from the largest
    index: a one-entry dictionary gets width 0). hybrid_decoder.go:83-85 returns 0 for every value
    without reading the stream, so the stream bytes after the width byte are arbitrary; here a few
    RLE and bit-packed run headers. Pages are long enough that every wave of a 4,096-value tile (and
    of a tile pair) has values. entries=0: every index is out of range (type_dict.go:52-54)."""
    rng = np.random.default_rng(1700 + seed)
    vocab = [int(x) for x in rng.integers(-2**31, 2**31 - 1, entries)]
    pages = [rawpq.dict_page_ref("INT32", vocab)]
    vals = []
    for nv in PAGE_VALUES:
        nulls = rng.random(nv) < (0.1 if optional else 0.0)
        dl = (~nulls).astype(int)
        body = bytes([0]) + rawpq.uvar(int(dl.sum()) << 1) + rawpq.uvar((3 << 1) | 1)
        pages.append(rawpq.data_page_v1_ref(nv, "RLE_DICTIONARY", body, dl.tolist() if optional else None,
                                            1 if optional else 0))
        vals += [vocab[0] if entries else None] * int(dl.sum())
    schema = [[(4, rawpq.BIN, "schema"), (5, rawpq.I32, 1)]]
    schema += [rawpq.schema_leaf("bw0", "INT32", "OPTIONAL" if optional else "REQUIRED")]
    return rawpq.write_file_schema(schema, [("bw0", "INT32")], [(sum(PAGE_VALUES), [(pages, sum(PAGE_VALUES), True)])]), vals


@pytest.mark.parametrize("optional", [False, True])
def test_oracle_dict_bw0(optional):
    data, expect = build_bw0(0, optional=optional)
    r = O.File(data).read_chunk(0, 0)
    np.testing.assert_array_equal(np.asarray(pqtest.oracle_values(r)), np.asarray(expect, np.int32))
    bad, _ = build_bw0(0, optional=optional, entries=0)
    with pytest.raises(O.OracleError) as e:
        O.File(bad).read_chunk(0, 0)
    assert (e.value.code, e.value.page) == (5, 0)  # PQ_ERR_DICT_INDEX on the first data page


@pytest.mark.gpu
@pytest.mark.parametrize("pair", ["1", "0"])
@pytest.mark.parametrize("optional", [False, True])
@pytest.mark.parametrize("entries", [1, 0])
def test_gpu_dict_bw0(gpu_ctx, pair, optional, entries, monkeypatch):
    """Bit width 0 on the early-dictionary path of do_dict (the one-entry dictionary is staged with
    the tile, and dict_tile_load ends without a barrier at width 0) and of do_dict2; decoded twice so
    that a read of stale LDS from an earlier workgroup would show."""
    import test_gpu_parity as P
    monkeypatch.setenv("PQ_DICT_PAIR", pair)
    data, _ = build_bw0(2, optional=optional, entries=entries)
    ((_, _, r),) = list(pqtest.oracle_decode(data))
    for rep in range(2):
        g = P._gpu_decode(gpu_ctx, data)[(0, 0)]
        where = f"pair={pair} optional={optional} entries={entries} rep={rep}"
        if isinstance(r, O.OracleError):
            assert isinstance(g, P.pqgpu.DecodeError), f"{where}: oracle error {r} but GPU decoded"
            assert (g.code, g.page) == (r.code, r.page), f"{where}: {g} vs {r}"
        else:
            assert not isinstance(g, P.pqgpu.DecodeError), f"{where}: GPU error {g}"
            pqtest.assert_chunk_equal(g, r, where)


@pytest.mark.gpu
@pytest.mark.parametrize("pair", ["1", "0"])
@pytest.mark.parametrize("optional", [False, True])
@pytest.mark.parametrize("bad", [False, True])
def test_gpu_dict_groups(gpu_ctx, pair, optional, bad, monkeypatch):
    import test_gpu_parity as P
    monkeypatch.setenv("PQ_DICT_PAIR", pair)  # 1: group every tile it can; 0: one tile per workgroup
    data, _ = build(1, bad=bad, optional=optional)
    gpu = P._gpu_decode(gpu_ctx, data)
    for rg, col, r in pqtest.oracle_decode(data):
        g = gpu[(rg, col)]
        where = f"pair={pair} optional={optional} bad={bad} {list(COLS)[col]}"
        if isinstance(r, O.OracleError):
            assert isinstance(g, P.pqgpu.DecodeError), f"{where}: oracle error {r} but GPU decoded"
            assert (g.code, g.page) == (r.code, r.page), f"{where}: {g} vs {r}"
        else:
            assert not isinstance(g, P.pqgpu.DecodeError), f"{where}: GPU error {g}"
            pqtest.assert_chunk_equal(g, r, where)
