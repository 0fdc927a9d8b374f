"""Flat OPTIONAL definition levels (bit width 1) through k_levels_seg (kernels.hip): the run-header
chain of every page is walked by 64 lanes from speculative starts, verified lane by lane, and
re-walked exactly where a lane's start was wrong or where a header needs the full decode
(hybrid_decoder.go:81-165 through decodePackedArray, helpers.go:133-149). These streams put the
speculation's hard cases at chosen places: Arrow-style alternating runs (what the lanes are tuned
for), the reference writer's single bit-packed run (a hop over every segment), long RLE runs,
non-minimal (5-byte) varint headers, payload bytes that are well-formed headers, streams longer
than the LDS stage and pages longer than the LDS bitmap, tiny streams, trailing garbage after
num_values, and every error class at a known value. The oracle (CPU restatement) gives the expected
levels, values and error; the GPU must equal it (the list-ranking kernel, PQ_LV_SEG=0, too)."""
import os
import struct
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import rawpq  # noqa: E402

import pqtest  # noqa: E402
import py_oracle as O  # noqa: E402


def uvar(x, pad=0):
    """uvarint of x, optionally padded with `pad` extra continuation bytes (non-minimal: Go's
    ReadUvarint accepts it)."""
    out = bytearray(rawpq.uvar(x))
    for _ in range(pad):
        out[-1] |= 0x80
        out.append(0)
    return bytes(out)


def rle(count, value, pad=0):
    return uvar(count << 1, pad) + bytes([value])


def lit(bits, pad=0):
    """one bit-packed run of len(bits) / 8 groups at bit width 1"""
    assert len(bits) % 8 == 0
    return uvar(((len(bits) // 8) << 1) | 1, pad) + np.packbits(np.asarray(bits, np.uint8), bitorder="little").tobytes()


def arrow_style(levels):
    """Arrow's RleEncoder shape: RLE runs for repeats of >= 8 aligned values, literal runs of at most
    63 groups otherwise (the run mix pyarrow writes for random nulls)."""
    out, i, n, pend = b"", 0, len(levels), []
    while i < n:
        j = i
        while j < n and levels[j] == levels[i]:
            j += 1
        if j - i >= 8 and (j == n or not pend):
            if pend:
                out += lit(pend)
                pend = []
            out += rle(j - i, int(levels[i]))
            i = j
            continue
        if n - i < 8:  # a partial last group: RLE runs instead of zero padding (streams concatenate)
            if pend:
                out += lit(pend)
                pend = []
            while i < n:
                j = i
                while j < n and levels[j] == levels[i]:
                    j += 1
                out += rle(j - i, int(levels[i]))
                i = j
            break
        pend += list(levels[i:i + 8])
        i += 8
        if len(pend) == 63 * 8:
            out += lit(pend)
            pend = []
    if pend:
        out += lit(pend)
    return out


def flat_file(pages, v2=False):
    """One INT32 OPTIONAL PLAIN column; pages = [(num_values, def stream bytes, non-null count)]."""
    out, total = [], 0
    for nv, st, nn in pages:
        vals = np.arange(nn, dtype="<i4").tobytes()
        if v2:
            dph = [(1, rawpq.I32, nv), (2, rawpq.I32, nv - nn), (3, rawpq.I32, nv), (4, rawpq.I32, 0),
                   (5, rawpq.I32, len(st)), (6, rawpq.I32, 0), (7, rawpq.BOOL, False)]
            out.append(rawpq._page(3, st + vals, 8, dph))
        else:
            dph = [(1, rawpq.I32, nv), (2, rawpq.I32, 0), (3, rawpq.I32, 3), (4, rawpq.I32, 3)]
            out.append(rawpq._page(0, struct.pack("<I", len(st)) + st + vals, 5, dph))
        total += nv
    schema = [[(4, rawpq.BIN, "schema"), (5, rawpq.I32, 1)], rawpq.schema_leaf("x", "INT32", "OPTIONAL")]
    return rawpq.write_file_schema(schema, [("x", "INT32")], [(total, [(out, total, False)])])


def random_levels(rng, n, null_frac):
    return (rng.random(n) >= null_frac).astype(np.uint8)


def good_pages(rng):
    """(num_values, stream, non-null count) pages whose streams decode without error."""
    pages = []
    for n, q in ((65_536, 0.1), (65_536, 0.5), (65_536, 0.02), (40_000, 0.1), (1_000, 0.1), (9, 0.3)):
        lv = random_levels(rng, n, q)
        pages.append((n, arrow_style(lv), int(lv.sum())))
    # the reference writer: one bit-packed run of the whole page (hybrid_encoder.go:55-70)
    lv = random_levels(rng, 65_536, 0.1)
    pages.append((65_536, rawpq.hybrid_ref(lv, 1), int(lv.sum())))
    # long RLE runs: all valid, all null, and a long null run between Arrow-style stretches
    pages.append((65_536, rle(65_536, 1), 65_536))
    pages.append((70_000, rle(70_000, 0), 0))
    lv = random_levels(rng, 60_000, 0.1)
    lv[20_000:45_000] = 0
    pages.append((60_000, arrow_style(lv), int(lv.sum())))
    # non-minimal varint headers (5 bytes: not the fast form) spread through an Arrow-style stream
    lv = random_levels(rng, 30_000, 0.1)
    st, parts = rle(16, 1, pad=4), [np.ones(16, np.uint8)]
    for k, cut in enumerate(range(2_000, 30_001, 2_000)):
        st += arrow_style(lv[cut - 2_000:cut])
        parts.append(lv[cut - 2_000:cut])
        if k % 3 == 0:  # a padded RLE run of 8 nulls, then a padded literal run
            st += rle(8, 0, pad=4) + lit([1, 0, 1, 1, 0, 1, 1, 1] * 4, pad=4)
            parts += [np.zeros(8, np.uint8), np.array([1, 0, 1, 1, 0, 1, 1, 1] * 4, np.uint8)]
    lvx = np.concatenate(parts)
    pages.append((len(lvx), st, int(lvx.sum())))
    # payload bytes that are themselves well-formed headers (0x03: a 1-group literal; 0x10: RLE 8)
    bits = np.unpackbits(np.frombuffer(bytes([0x03, 0x10, 0x01, 0x05]) * 2_000, np.uint8), bitorder="little")
    chunks = [lit(bits[k:k + 504]) for k in range(0, len(bits) - 504, 504)]
    st = b"".join(c + rle(9, 1) for c in chunks)
    lvx = np.concatenate([np.concatenate([bits[k:k + 504], np.ones(9, np.uint8)]) for k in range(0, len(bits) - 504, 504)])
    pages.append((len(lvx), st, int(lvx.sum())))
    # a stream longer than the LDS stage and a page longer than the LDS bitmap (300,000 slots)
    lv = random_levels(rng, 300_000, 0.1)
    pages.append((300_000, arrow_style(lv), int(lv.sum())))
    # trailing bytes after the run that reaches num_values (never read): garbage and an empty run
    lv = random_levels(rng, 20_000, 0.1)
    pages.append((20_000, arrow_style(lv) + bytes([0x00, 0x00, 0xff, 0xff, 0xff, 0xff, 0xff]), int(lv.sum())))
    # num_values ending inside a run
    lv = random_levels(rng, 20_000, 0.1)
    pages.append((19_995, arrow_style(lv), int(lv[:19_995].sum())))
    return pages


def bad_pages(rng):
    """Pages that fail, each with one error at a known place (the previous page is valid)."""
    lv = random_levels(rng, 30_000, 0.1)
    a = arrow_style(lv[:15_000])
    b = arrow_style(lv[15_000:])
    out = []
    out.append((30_000, a + rle(0, 1) + b, 0))               # empty run: "rle: empty run"
    out.append((30_000, a + rle(16, 2) + b, 0))              # RLE value >= 2^bw
    out.append((30_000, a + b[: len(b) // 2], 0))            # stream ends before num_values (EOF)
    out.append((30_000, a + lit([1] * 800)[:60], 0))          # a bit-packed run cut by EOF
    out.append((30_000, a + bytes([0xff] * 20), 0))           # a varint that never ends (overflow / EOF)
    out.append((30_000, a + rle(16, 1)[:1], 0))               # RLE value missing (EOF)
    return out


@pytest.fixture(scope="module")
def files():
    rng = np.random.default_rng(41)
    good = good_pages(rng)
    out = {"good_v1": flat_file(good), "good_v2": flat_file(good, v2=True)}
    ok = good[0]
    for k, p in enumerate(bad_pages(rng)):
        out[f"bad{k}"] = flat_file([ok, p])
    return out


def test_oracle_levels_streams(files):
    """The restatement accepts the good streams (levels equal what was encoded) and fails each bad
    page with an error on page 1."""
    for name, data in files.items():
        for _rg, _col, r in pqtest.oracle_decode(data):
            if name.startswith("good"):
                assert not isinstance(r, O.OracleError), (name, r)
            else:
                assert isinstance(r, O.OracleError) and r.page == 1, (name, r)
    rng = np.random.default_rng(41)
    good = good_pages(rng)
    (_, _, r), = pqtest.oracle_decode(files["good_v1"])
    assert r.num_values == sum(nn for _, _, nn in good)


@pytest.mark.gpu
@pytest.mark.parametrize("kernel", ["seg", "seg_grid1", "ranking"])
def test_gpu_levels_streams(gpu_ctx, files, monkeypatch, kernel):
    """seg_grid1: one k_levels_seg wavefront walks every page in turn (a wave's second and later pages
    reuse its LDS stage and bitmap image)."""
    import pqgpu
    import test_gpu_parity as P
    if kernel == "ranking":
        monkeypatch.setenv("PQ_LV_SEG", "0")
    if kernel == "seg_grid1":
        monkeypatch.setenv("PQ_SEG_GRID", "1")
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
