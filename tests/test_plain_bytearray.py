"""PLAIN BYTE_ARRAY pages (byteArrayPlainDecoder, type_bytearray.go:24-55) through the parallel
length-chain walk (plainba.hip: speculative 256-byte segments, verified per page). The page
shapes are chosen to defeat the speculation — binary payloads whose bytes read as plausible
lengths, runs of empty values (every position of a zero run looks like a value start), payloads
that embed well-formed [length | bytes] chains, values longer than a segment — and to hit every
error of the reference's value loop (negative length, short length, short payload, too few
values for the header's count) at a known value, plus trailing bytes after the last counted
value (never read by the reference). The GPU must equal the oracle."""
import os
import struct
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import rawpq  # noqa: E402

import pqtest  # noqa: E402
import py_oracle as O  # noqa: E402


def _values(rng, kind, n):
    if kind == "binary":
        return [rng.integers(0, 256, int(rng.integers(0, 41)), dtype=np.uint8).tobytes() for _ in range(n)]
    if kind == "text":
        return [bytes(rng.integers(97, 123, int(rng.integers(1, 30)), dtype=np.uint8)) for _ in range(n)]
    if kind == "empty":  # long runs of zero lengths between a few values
        return [b"" if rng.random() < 0.9 else b"xyz" for _ in range(n)]
    if kind == "embedded":  # payloads that are themselves [u32 len | bytes] chains
        out = []
        for _ in range(n):
            inner = b"".join(struct.pack("<I", k) + b"q" * k for k in rng.integers(0, 6, 4))
            out.append(inner)
        return out
    if kind == "long":  # values spanning several segments
        return [bytes([int(rng.integers(1, 255))]) * int(rng.choice([3, 300, 1000, 5000])) for _ in range(n)]
    if kind == "smallints":  # bytes that read as small little-endian lengths almost everywhere
        return [bytes(rng.integers(0, 3, int(rng.integers(0, 24)), dtype=np.uint8)) for _ in range(n)]
    raise ValueError(kind)


def _section(vals):
    return b"".join(struct.pack("<I", len(v)) + v for v in vals)


def build(seed, kinds=("binary", "text", "empty", "embedded", "long", "smallints"), pages=3, n=3000):
    """One REQUIRED BYTE_ARRAY column per kind, `pages` PLAIN V1 pages each."""
    rng = np.random.default_rng(900 + seed)
    chunks = []
    for kind in kinds:
        ps, tot = [], 0
        for _ in range(pages):
            m = int(rng.integers(1, n))
            ps.append(rawpq.data_page_v1_ref(m, "PLAIN", _section(_values(rng, kind, m))))
            tot += m
        chunks.append((ps, tot))
    return _file(kinds, chunks)


def _file(names, chunks):
    """One row group; chunks: [(page byte strings, total num_values)] per REQUIRED BYTE_ARRAY column."""
    schema = [[(4, rawpq.BIN, "schema"), (5, rawpq.I32, len(names))]]
    schema += [rawpq.schema_leaf(name, "BYTE_ARRAY", "REQUIRED") for name in names]
    leaves = [(name, "BYTE_ARRAY") for name in names]
    return rawpq.write_file_schema(schema, leaves, [(max(nv for _, nv in chunks), [(ps, nv, False) for ps, nv in chunks])])


def bad_pages(seed=0):
    """Pages that fail at a known value, and one with trailing bytes after its last value."""
    rng = np.random.default_rng(950 + seed)
    good = _values(rng, "text", 1500)
    sec = _section(good)
    cases = {}
    # negative length at value 1000
    neg = _section(good[:1000]) + struct.pack("<i", -5) + b"abcde" + _section(good[1000:])
    cases["negative"] = (neg, 1500, (3, 1000))
    # payload cut short inside value 1499
    cases["short_payload"] = (sec[:-3], 1500, (2, 1499))
    # length cut short: 2 bytes of value 1500's length
    cases["short_length"] = (sec + b"\x07\x00", 1501, (2, 1500))
    # the header counts more values than the section holds: io.EOF at value 1500
    cases["too_few"] = (sec, 1510, (1, 1500))
    # trailing bytes after the 1500 counted values: never read
    cases["trailing"] = (sec + b"\xff\xff\xff\x7f" + b"junk" * 100, 1500, None)
    # an empty section with values expected
    cases["empty_section"] = (b"", 4, (1, 0))
    # a value whose length reaches exactly the section end, then EOF
    cases["exact_end_then_eof"] = (sec, 1501, (1, 1500))
    return cases


def _oracle_and_gpu(gpu_ctx, data):
    import test_gpu_parity as P
    return pqtest.oracle_decode(data), P._gpu_decode(gpu_ctx, data)


def test_oracle_plain_values():
    rng = np.random.default_rng(1)
    for kind in ("binary", "text", "empty", "embedded", "long", "smallints"):
        vals = _values(rng, kind, 200)
        data = _file([kind], [([rawpq.data_page_v1_ref(len(vals), "PLAIN", _section(vals))], len(vals))])
        r = O.File(data).read_chunk(0, 0)
        assert pqtest.oracle_values(r) == vals, kind


def test_oracle_bad_pages():
    for name, (sec, nv, want) in bad_pages().items():
        data = _file([name], [([rawpq.data_page_v1_ref(nv, "PLAIN", sec)], nv)])
        try:
            O.File(data).read_chunk(0, 0)
            got = None
        except O.OracleError as e:
            got = e.code
        assert got == (None if want is None else want[0]), (name, got, want)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [0, 1, 2])
def test_gpu_plain_bytearray(gpu_ctx, seed):
    data = build(seed)
    orc, gpu = _oracle_and_gpu(gpu_ctx, data)
    kinds = ("binary", "text", "empty", "embedded", "long", "smallints")
    for rg, col, r in orc:
        assert not isinstance(r, O.OracleError), (kinds[col], r)
        pqtest.assert_chunk_equal(gpu[(rg, col)], r, f"seed={seed} {kinds[col]}")


@pytest.mark.gpu
def test_gpu_plain_bytearray_errors(gpu_ctx):
    import pqgpu
    cases = bad_pages()
    names = list(cases)
    chunks = [([rawpq.data_page_v1_ref(5, "PLAIN", _section([b"ok"] * 5)),
                rawpq.data_page_v1_ref(nv, "PLAIN", sec)], 5 + nv)
              for sec, nv, _want in cases.values()]
    data = _file(names, chunks)
    orc, gpu = _oracle_and_gpu(gpu_ctx, data)
    for rg, col, r in orc:
        g = gpu[(rg, col)]
        want = cases[names[col]][2]
        if isinstance(r, O.OracleError):
            assert want is not None and (r.code, r.page) == (want[0], 1), (names[col], r)
            assert isinstance(g, pqgpu.DecodeError) and (g.code, g.page) == (r.code, r.page), (names[col], g, r)
        else:
            assert want is None, names[col]
            pqtest.assert_chunk_equal(g, r, names[col])
