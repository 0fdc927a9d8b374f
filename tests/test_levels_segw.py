"""Generic level streams (repetition levels of bit width 1, definition levels of bit width 2) through
k_levels_segw (kernels.hip): one 512-lane workgroup per (page, stream) walks its segments from
speculative starts, verifies them in lane order across its waves, re-walks failing lanes exactly and
writes the stream's run table for k_level_fill (hybrid_decoder.go:81-165 through decodePackedArray,
helpers.go:133-149; page_v1.go:33-63). The column is `l: optional group (LIST) { repeated group list
{ optional int32 element } }` (maxR 1, maxD 3), records drawn at random (null lists, empty lists,
null elements). The streams are Arrow-style run mixes, the reference writer's single bit-packed run,
long runs, non-minimal varint headers, a stream longer than the workgroup's LDS stage (the
list-ranking kernel takes it), num_values ending inside a run, and errors at known values in either
stream. The oracle gives levels, values and errors; the GPU must equal it on every level-kernel route
(k_levels_segw, k_levels_hyb, k_levels)."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import rawpq  # noqa: E402

import pqtest  # noqa: E402
import py_oracle as O  # noqa: E402
from test_levels_seg import uvar  # noqa: E402


def rle(count, value, bw, pad=0):
    return uvar(count << 1, pad) + int(value).to_bytes((bw + 7) // 8, "little")


def lit(vals, bw, pad=0):
    assert len(vals) % 8 == 0
    return uvar(((len(vals) // 8) << 1) | 1, pad) + rawpq.bitpack([int(v) for v in vals], bw)


def arrow_style(levels, bw):
    """RLE runs for repeats of >= 8 values, literal runs of at most 63 groups otherwise; a partial
    last group as RLE runs (so streams concatenate)."""
    out, i, n, pend = b"", 0, len(levels), []
    while i < n:
        j = i
        while j < n and levels[j] == levels[i]:
            j += 1
        if j - i >= 8 and not pend:
            out += rle(j - i, levels[i], bw)
            i = j
            continue
        if n - i < 8:
            if pend:
                out += lit(pend, bw)
                pend = []
            while i < n:
                j = i
                while j < n and levels[j] == levels[i]:
                    j += 1
                out += rle(j - i, levels[i], bw)
                i = j
            break
        pend += list(levels[i:i + 8])
        i += 8
        if len(pend) == 63 * 8:
            out += lit(pend, bw)
            pend = []
    if pend:
        out += lit(pend, bw)
    return out


def records(rng, nrec):
    """(rep, def) levels of nrec random records of the list column."""
    rep, dfn = [], []
    for _ in range(nrec):
        u = rng.random()
        if u < 0.05:
            rep.append(0); dfn.append(0)  # null list
        elif u < 0.10:
            rep.append(0); dfn.append(1)  # empty list
        else:
            k = int(rng.integers(1, 9))
            for e in range(k):
                rep.append(0 if e == 0 else 1)
                dfn.append(3 if rng.random() >= 0.05 else 2)
    return np.array(rep, np.uint8), np.array(dfn, np.uint8)


def list_file(pages):
    """pages: [(num_values, rep stream, def stream, non-null count)] as DATA_PAGE (V1) pages."""
    import struct
    out, total = [], 0
    for nv, rs, ds, nn in pages:
        body = struct.pack("<I", len(rs)) + rs + struct.pack("<I", len(ds)) + ds + np.arange(nn, dtype="<i4").tobytes()
        dph = [(1, rawpq.I32, nv), (2, rawpq.I32, 0), (3, rawpq.I32, 3), (4, rawpq.I32, 3)]
        out.append(rawpq._page(0, body, 5, dph))
        total += nv
    G, L = rawpq.schema_group, rawpq.schema_leaf
    schema = [[(4, rawpq.BIN, "schema"), (5, rawpq.I32, 1)], G("l", "OPTIONAL", 1) + [(6, rawpq.I32, 3)],
              G("list", "REPEATED", 1), L("element", "INT32", "OPTIONAL")]
    return rawpq.write_file_schema(schema, [("l.list.element", "INT32")], [(1, [(out, total, False)])])


def page(rep, dfn, rs=None, ds=None, nv=None):
    nv = len(rep) if nv is None else nv
    return (nv, arrow_style(rep, 1) if rs is None else rs, arrow_style(dfn, 2) if ds is None else ds,
            int((dfn[:nv] == 3).sum()))


def good_pages(rng):
    pages = []
    for nrec in (14_000, 3_000, 200, 1):
        r, d = records(rng, nrec)
        pages.append(page(r, d))
    r, d = records(rng, 9_000)  # the reference writer: one bit-packed run per stream
    pages.append(page(r, d, rawpq.hybrid_ref(r, 1), rawpq.hybrid_ref(d, 2)))
    # long runs: 40,000 one-element records with present elements, then 5,000 null lists
    r = np.concatenate([np.zeros(40_000, np.uint8), np.zeros(5_000, np.uint8)])
    d = np.concatenate([np.full(40_000, 3, np.uint8), np.zeros(5_000, np.uint8)])
    pages.append(page(r, d))
    # non-minimal (5-byte) varint headers between Arrow-style stretches
    r, d = records(rng, 6_000)
    k = len(r) // 2
    rs = arrow_style(r[:k], 1) + rle(8, 0, 1, pad=4) + arrow_style(r[k:], 1)
    ds = arrow_style(d[:k], 2) + rle(8, 1, 2, pad=4) + arrow_style(d[k:], 2)
    pages.append((len(r) + 8, rs, ds, int((d == 3).sum())))
    # longer than the workgroup's stage (the list-ranking kernel takes the definition stream)
    r, d = records(rng, 70_000)
    pages.append(page(r, d))
    # num_values ending inside a run, trailing garbage after it
    r, d = records(rng, 5_000)
    pages.append(page(r, d, arrow_style(r, 1) + b"\x00\xff\xff\xff\xff", arrow_style(d, 2) + b"\x00\x00", nv=len(r) - 3))
    return pages


def bad_pages(rng):
    r, d = records(rng, 8_000)
    h = len(r) // 2
    ra, rb = arrow_style(r[:h], 1), arrow_style(r[h:], 1)
    da, db = arrow_style(d[:h], 2), arrow_style(d[h:], 2)
    n = len(r)
    return [
        (n, ra + rb, da + rle(16, 5, 2) + db, 0),      # RLE definition value >= 2^bw
        (n, ra + rle(0, 0, 1) + rb, da + db, 0),        # empty repetition run
        (n, ra + rb, da + db[: len(db) // 3], 0),       # definition stream ends early (EOF)
        (n, ra + rb, da + lit([3] * 800, 2)[:90], 0),   # a bit-packed run cut by EOF
        (n, ra + rb[:7], da + db, 0),                   # repetition stream ends early
    ]


@pytest.fixture(scope="module")
def files():
    rng = np.random.default_rng(77)
    good = good_pages(rng)
    out = {"good": list_file(good)}
    for k, p in enumerate(bad_pages(rng)):
        out[f"bad{k}"] = list_file([good[1], p])
    return out


def test_oracle_generic_streams(files):
    for name, data in files.items():
        for _rg, _col, r in pqtest.oracle_decode(data):
            if name == "good":
                assert not isinstance(r, O.OracleError), (name, r)
            else:
                assert isinstance(r, O.OracleError) and r.page == 1, (name, r)


# level-kernel routes (host.cpp): "seg" every stream by k_levels_segw; "ranking" every stream by
# k_levels (its stride prelude takes the repetition streams' literal runs); "hyb" repetition streams by
# k_levels_hyb, definition streams by k_levels; "default" definition streams by k_levels_segw,
# repetition streams by k_levels_hyb
ROUTES = {"seg": {"PQ_LV_SEGW": "1"}, "ranking": {"PQ_LV_SEGW": "0", "PQ_LV_HYB": "0"},
          "hyb": {"PQ_LV_SEGW": "0"}, "default": {}}


@pytest.mark.gpu
@pytest.mark.parametrize("kernel", list(ROUTES))
def test_gpu_generic_streams(gpu_ctx, files, monkeypatch, kernel):
    import pqgpu
    import test_gpu_parity as P
    for k in ("PQ_LV_SEGW", "PQ_LV_HYB"):
        monkeypatch.delenv(k, raising=False)
    for k, v in ROUTES[kernel].items():
        monkeypatch.setenv(k, v)
    for name, data in files.items():
        gpu = P._gpu_decode(gpu_ctx, data)
        for rg, col, r in pqtest.oracle_decode(data):
            g = gpu[(rg, col)]
            if isinstance(r, O.OracleError):
                assert isinstance(g, pqgpu.DecodeError), (name, g)
                assert (g.code, g.page) == (r.code, r.page), (name, g, r)
            else:
                assert not isinstance(g, pqgpu.DecodeError), (name, g)
                pqtest.assert_chunk_equal(g, r, f"{name} ({kernel})")
