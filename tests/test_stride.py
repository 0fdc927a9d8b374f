"""Hand-built hybrid and DELTA streams for the stride speculation of the run-header walks
(kernels.hip hyb_scan: dictionary-index runs of one header back to back; do_delta_page: blocks
of one length back to back). A lane takes the header k runs (blocks) ahead as if the runs between
had the current header; only the leading lanes whose header repeats are trusted. These streams
put the places where that stops — a different run, the end of the page's values inside a stride,
the stream ending inside a run, the LDS window boundary — at chosen positions. The oracle
(hybrid_decoder.go:81-165, deltabp_decoder.go:113-174 restated) gives the expected values and
error; the GPU must equal it."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import rawpq  # noqa: E402

import pqtest  # noqa: E402
import py_oracle as O  # noqa: E402


def lit(vals, bw):
    """One bit-packed run of len(vals) / 8 groups."""
    assert len(vals) % 8 == 0
    return rawpq.uvar(((len(vals) // 8) << 1) | 1) + rawpq.bitpack([int(v) for v in vals], bw)


def rle(count, value, bw):
    return rawpq.uvar(count << 1) + int(value).to_bytes((bw + 7) // 8, "little")


def dict_file(pages, dict_size, bw):
    """One INT32 REQUIRED RLE_DICTIONARY column: pages = [(num_values, run bytes)]."""
    rng = np.random.default_rng(7)
    d = rng.integers(-2**31, 2**31 - 1, dict_size, dtype=np.int64).astype(np.int32)
    out = [rawpq.dict_page_ref("INT32", d)]
    n = 0
    for nv, runs in pages:
        out.append(rawpq.data_page_v1_ref(nv, "RLE_DICTIONARY", bytes([bw]) + runs))
        n += nv
    schema = [[(4, rawpq.BIN, "schema"), (5, rawpq.I32, 1)], rawpq.schema_leaf("x", "INT32", "REQUIRED")]
    return rawpq.write_file_schema(schema, [("x", "INT32")], [(n, [(out, n, True)])])


def index_pages(bw, rng):
    hi = 1 << bw
    full = lambda: rng.integers(0, hi, 504)  # 63 groups: the longest literal run of a 1-byte header
    pages = []
    # 1. 40 equal literal runs: strides across the 16 KiB window boundary (bw 8: 505 B per run)
    runs = b"".join(lit(full(), bw) for _ in range(40))
    pages.append((40 * 504, runs))
    # 2. the same runs, num_values ending inside the second stride and inside a run
    pages.append((10_001, runs))
    # 3. equal runs broken by a shorter literal run, an RLE run, then equal runs again
    r3 = b"".join(lit(full(), bw) for _ in range(9)) + lit(rng.integers(0, hi, 80), bw) + rle(300, hi - 1, bw)
    r3 += b"".join(lit(full(), bw) for _ in range(12))
    pages.append((9 * 504 + 80 + 300 + 12 * 504, r3))
    # 4. alternating run lengths (no stride longer than one run)
    r4 = b"".join(lit(rng.integers(0, hi, 504 if k % 2 else 496), bw) for k in range(20))
    pages.append((10 * 504 + 10 * 496, r4))
    # 5. payload bytes equal to the run header everywhere (index 127 at bw 8: 0x7f)
    r5 = b"".join(lit(np.full(504, 127 if bw == 8 else 0x7f7f), bw) for _ in range(30))
    pages.append((30 * 504, r5))
    # 6. short runs: RLE runs of 1-3 values and 1-group literal runs, > 256 runs per 4096-value
    # tile (k_values_dict keeps 256 runs in LDS and reads a longer tile's runs from global memory)
    r6, n6 = b"", 0
    for k in range(4000):
        if k % 5 == 4:
            r6 += lit(rng.integers(0, hi, 8), bw)
            n6 += 8
        else:
            r6 += rle(1 + k % 3, (k * 7) % hi, bw)
            n6 += 1 + k % 3
    pages.append((n6, r6))
    return pages


@pytest.mark.parametrize("bw,dict_size", [(8, 256), (16, 65536)])
def test_oracle_stride_streams(bw, dict_size):
    rng = np.random.default_rng(bw)
    data = dict_file(index_pages(bw, rng), dict_size, bw)
    (_, _, r), = pqtest.oracle_decode(data)
    assert not isinstance(r, O.OracleError), r
    assert r.num_values == sum(nv for nv, _ in index_pages(bw, np.random.default_rng(bw)))


def truncated_file(bw, cut):
    """Equal literal runs whose stream ends `cut` bytes before the last run's end: a group that
    starts before the end is zero-filled (hybrid_decoder.go:132-140), the first group that does not
    fails the page with io.EOF at its first value."""
    rng = np.random.default_rng(3)
    runs = b"".join(lit(rng.integers(0, 1 << bw, 504), bw) for _ in range(30))
    return dict_file([(4 * 504, runs[:4 * (len(runs) // 30)]), (30 * 504, runs[:-cut])], 1 << bw, bw)


@pytest.mark.parametrize("cut", [1, 100, 504])
def test_oracle_stride_truncated(cut):
    (_, _, r), = pqtest.oracle_decode(truncated_file(8, cut))
    if cut < 8:  # the last group starts before the end: zero-filled, no error
        assert not isinstance(r, O.OracleError), r
    else:
        assert isinstance(r, O.OracleError) and r.page == 1, r


def delta_file(page_vals, bs=128, mbc=4):
    return rawpq.delta_column_file(page_vals, bs, mbc, typ="INT64")


def delta_pages(rng):
    steady = lambda n: np.cumsum(rng.integers(0, 2**16, n))  # miniblock widths 16: equal blocks
    pages = [steady(60_000), steady(1_000)]
    # a block of different widths in the middle of equal ones, then equal blocks again
    a = steady(20_000)
    a[7_000:7_128] = np.cumsum(rng.integers(0, 2**40, 128)) + a[6_999]
    a[7_128:] += a[7_127] - a[7_128] + 5
    pages.append(a)
    return [[int(x) for x in p] for p in pages]


def test_oracle_stride_delta():
    data = delta_file(delta_pages(np.random.default_rng(11)))
    for _, _, r in pqtest.oracle_decode(data):
        assert not isinstance(r, O.OracleError), r


@pytest.mark.gpu
@pytest.mark.parametrize("bw,dict_size", [(8, 256), (16, 65536)])
def test_gpu_stride_streams(gpu_ctx, bw, dict_size):
    import test_gpu_parity as P
    data = dict_file(index_pages(bw, np.random.default_rng(bw)), dict_size, bw)
    gpu = P._gpu_decode(gpu_ctx, data)
    for rg, col, r in pqtest.oracle_decode(data):
        pqtest.assert_chunk_equal(gpu[(rg, col)], r, f"bw {bw}")


@pytest.mark.gpu
@pytest.mark.parametrize("cut", [1, 100, 504])
def test_gpu_stride_truncated(gpu_ctx, cut):
    import pqgpu
    import test_gpu_parity as P
    data = truncated_file(8, cut)
    gpu = P._gpu_decode(gpu_ctx, data)
    (rg, col, r), = pqtest.oracle_decode(data)
    g = gpu[(rg, col)]
    if isinstance(r, O.OracleError):
        assert isinstance(g, pqgpu.DecodeError), g
        assert (g.code, g.page) == (r.code, r.page), (g, r)
    else:
        assert not isinstance(g, pqgpu.DecodeError), g
        pqtest.assert_chunk_equal(g, r, f"cut {cut}")


@pytest.mark.gpu
def test_gpu_stride_delta(gpu_ctx):
    import test_gpu_parity as P
    data = delta_file(delta_pages(np.random.default_rng(11)))
    gpu = P._gpu_decode(gpu_ctx, data)
    for rg, col, r in pqtest.oracle_decode(data):
        pqtest.assert_chunk_equal(gpu[(rg, col)], r, "delta")
