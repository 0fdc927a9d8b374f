"""DELTA_BINARY_PACKED stream shapes pyarrow never writes (tools/rawpq.py builds them
from the format specification): block sizes 128..2048 and 384, 1..16 miniblocks
(mbc > 8 and miniblocks of 4 values take the exact scalar path), widths 0..64,
non-zero widths in unused trailing miniblocks, N = 1 mod block
size (Q1), truncated payloads, INT32 wrap-around. The oracle must return the
generator's values (or the reference's error); the GPU must equal the oracle."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import rawpq  # noqa: E402

import pqtest  # noqa: E402
import py_oracle as O  # noqa: E402

SHAPES = [  # (block size, miniblocks, step bits, typ)
    (128, 4, 7, "INT64"), (256, 4, 16, "INT64"), (256, 8, 33, "INT64"), (512, 4, 3, "INT64"),
    (1024, 8, 20, "INT64"), (2048, 8, 12, "INT64"), (2048, 1, 63, "INT64"), (128, 1, 9, "INT64"),
    (384, 4, 10, "INT64"), (128, 16, 5, "INT64"), (128, 32, 5, "INT64"),
    (256, 4, 31, "INT32"), (128, 4, 32, "INT32"), (512, 2, 1, "INT32"), (256, 16, 4, "INT32"),
    # more than 256 miniblocks per block: valid streams the reference decodes (widths are read
    # in place by the exact scalar path, no per-block width buffer)
    (4096, 512, 9, "INT64"), (8192, 1024, 5, "INT32"),
]
COUNTS = [2, 8, 9, 100, 129, 255, 256, 258, 1000, 2047, 2049, 5000, 20000]


def _values(rng, n, step_bits, typ):
    v = rawpq.random_walk(rng, n, step_bits)
    if typ == "INT32":
        v = [((x + 2**31) % 2**32) - 2**31 for x in v]
    return v


def _shape_file(k, bs, mbc, step, typ, trailing=0):
    rng = np.random.default_rng(100 + k)
    counts = [c for c in COUNTS if c % bs != 1]  # N = 1 (mod bs): Q1, tested below
    pages = [_values(rng, c, step, typ) for c in counts]
    return rawpq.delta_column_file(pages, bs, mbc, typ=typ, v2=k % 2 == 1, rg_split=[len(pages) // 2, len(pages) - len(pages) // 2],
                                   trailing_width=trailing), pages


def _gpu_chunks(ctx, data):
    import pqgpu
    f = pqgpu.File(data)
    b = pqgpu.Batch(ctx)
    ids = [(rg, b.add_file_chunk(f, rg, 0)[0]) for rg in range(f.num_row_groups)]
    b.decode()
    b.sync()
    out = {rg: (b.status(cid) or b.result(cid)) for rg, cid in ids}
    b.close()
    return out


@pytest.mark.parametrize("k", range(len(SHAPES)))
def test_oracle_delta_shapes(k):
    bs, mbc, step, typ = SHAPES[k]
    if (bs // mbc) % 8:
        pytest.skip("miniblocks of 4 values: the reference reads 8 at a time across them (GPU test compares errors)")
    data, pages = _shape_file(k, bs, mbc, step, typ)  # trailing widths 0: every page decodes
    f = O.File(data)
    got = np.concatenate([np.asarray(f.read_chunk(rg, 0).values) for rg in range(f.num_row_groups)])
    want = np.asarray([x for p in pages for x in p], np.int64 if typ == "INT64" else np.int32)
    assert np.array_equal(got, want)


@pytest.mark.gpu
@pytest.mark.parametrize("k", range(len(SHAPES)))
def test_gpu_delta_shapes(gpu_ctx, k):
    bs, mbc, step, typ = SHAPES[k]
    for trailing in (0, (k * 7) % 17 + 1):
        # non-zero widths in unused trailing miniblocks: the look-ahead (Q1) reads a group
        # the writer never emitted whenever delta N-1 opens such a miniblock -> io.EOF
        data, _ = _shape_file(k, bs, mbc, step, typ, trailing=trailing)
        orc = O.File(data)
        gpu = _gpu_chunks(gpu_ctx, data)
        for rg in range(orc.num_row_groups):
            where = f"shape {SHAPES[k]} trailing {trailing} rg{rg}"
            try:
                want = orc.read_chunk(rg, 0)
            except O.OracleError as e:
                assert (gpu[rg].code, gpu[rg].page) == (e.code, e.page), (where, gpu[rg], e)
                continue
            pqtest.assert_chunk_equal(gpu[rg], want, where)


@pytest.mark.gpu
@pytest.mark.parametrize("bs,n", [(256, 257), (128, 129), (256, 513), (2048, 2049), (128, 1025)])
def test_gpu_delta_q1_lookahead(gpu_ctx, bs, n):
    """N = 1 (mod block size): value N-1 reads a block header no writer emits -> io.EOF there."""
    rng = np.random.default_rng(n)
    data = rawpq.delta_column_file([_values(rng, n, 12, "INT64")], bs, 4)
    with pytest.raises(O.OracleError) as e:
        O.File(data).read_chunk(0, 0)
    g = _gpu_chunks(gpu_ctx, data)[0]
    assert g.code == e.value.code == 1 and g.page == e.value.page == 0


@pytest.mark.gpu
@pytest.mark.parametrize("cut", [1, 7, 50, 301, 1000])
def test_gpu_delta_truncated(gpu_ctx, cut):
    """A DELTA page whose stream is cut: the first unreadable group / header fails the page
    with the reference's error class at the same page (or, when only padding was cut, the
    page decodes as in the reference)."""
    rng = np.random.default_rng(cut)
    vals = _values(rng, 4000, 14, "INT64")
    st = rawpq.delta_encode(vals, 256, 4, 64)
    st = st[: len(st) - cut]
    page = rawpq.page_v1(st, len(vals), "DELTA_BINARY_PACKED")
    data = rawpq.write_file([("a", "INT64", False)], [(len(vals), [[page]], [len(vals)])])
    try:
        O.File(data).read_chunk(0, 0)
        orc_err = None
    except O.OracleError as e:
        orc_err = e
    g = _gpu_chunks(gpu_ctx, data)[0]
    if orc_err is None:  # the cut only removed padding the decoder never reads
        pqtest.assert_chunk_equal(g, O.File(data).read_chunk(0, 0), f"cut {cut}")
    else:
        assert (g.code, g.page) == (orc_err.code, orc_err.page)
