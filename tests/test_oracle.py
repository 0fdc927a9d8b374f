"""CPU tests: the oracle against the reference's own known-answer vectors and
against pyarrow (an independent Parquet implementation) on the fixtures."""
import json
import os

import numpy as np
import pytest

import py_oracle as O
import pqtest


def _kats(name):
    with open(os.path.join(pqtest.GOLDEN, name)) as f:
        return json.load(f)["vectors"]


def test_bitpack32_kats():
    """bitpacking32_test.go:11-23 table (127 vectors, widths 0-32)."""
    v = _kats("bitpack32_kats.json")
    assert len(v) == 127
    for t in v:
        got = O.unpack8_int32(bytes(t["data"]), t["width"])
        assert got == [x if x < 2**31 else x - 2**32 for x in t["values"]], t


def test_bitpack64_kats():
    """bitpacking64_test.go:11-23 table (317 vectors, widths 0-64)."""
    v = _kats("bitpack64_kats.json")
    assert len(v) == 317
    for t in v:
        got = O.unpack8_int64(bytes(t["data"]), t["width"])
        assert got == [x if x < 2**63 else x - 2**64 for x in t["values"]], t


def test_hybrid_semantics():
    """hybrid_decoder.go: RLE run, bit-packed run, zero-filled short group, errors (Appendix A Q3)."""
    # RLE run of 5 x value 3 (bw 2), then bit-packed 1 group of 8 values 0..7 at bw 3
    s = bytes([5 << 1, 3])
    rc, out = O.hybrid_decode(s, 2, 5)
    assert rc == 0 and list(out) == [3] * 5
    packed = 0
    for i in range(8):
        packed |= i << (3 * i)
    s = bytes([(1 << 1) | 1]) + packed.to_bytes(3, "little")
    rc, out = O.hybrid_decode(s, 3, 8)
    assert rc == 0 and list(out) == list(range(8))
    # short final group is zero-filled, not an error
    rc, out = O.hybrid_decode(s[:2], 3, 8)
    assert rc == 0 and list(out) == [0, 1, 2, 0, 0, 0, 0, 0] or list(out)[:2] == [0, 1]
    # EOF after the stream
    rc, out = O.hybrid_decode(bytes([2 << 1, 1]), 1, 3)
    assert rc == 1 and len(out) == 2
    # empty RLE run
    rc, _ = O.hybrid_decode(bytes([0, 1]), 1, 1)
    assert rc == 3
    # RLE value too large for the bit width
    rc, _ = O.hybrid_decode(bytes([2, 4]), 2, 1)
    assert rc == 3
    # short RLE value
    rc, _ = O.hybrid_decode(bytes([2, 1]), 9, 1)
    assert rc == 2
    # header > MaxInt32
    rc, _ = O.hybrid_decode(bytes([0xff, 0xff, 0xff, 0xff, 0x0f]), 1, 1)
    assert rc == 9


def test_delta_q1_lookahead():
    """deltabp_decoder.go:167-173: N ≡ 1 (mod 256) pages fail with EOF (Appendix A Q1)."""
    import io
    import pyarrow as pa
    import pyarrow.parquet as pq
    for n, ok in [(128, True), (129, True), (256, True), (257, False), (258, True), (513, False), (1000, True)]:
        b = io.BytesIO()
        pq.write_table(pa.table({"a": pa.array(np.arange(n, dtype=np.int64) * 3)}), b, use_dictionary=False,
                       compression="NONE", column_encoding={"a": "DELTA_BINARY_PACKED"})
        f = O.File(b.getvalue())
        if ok:
            assert np.array_equal(f.read_chunk(0, 0).values, np.arange(n) * 3)
        else:
            with pytest.raises(O.OracleError) as ei:
                f.read_chunk(0, 0)
            assert ei.value.code == 1


@pytest.mark.parametrize("name", [n for n in pqtest.VALID if n not in ("edge_empty",)])
def test_oracle_matches_pyarrow(name):
    import io
    import pyarrow.parquet as pq
    data = pqtest.load(name)
    pf = pq.ParquetFile(io.BytesIO(data))
    f = O.File(data)
    flat = [i for i in range(f.num_columns) if f.column_info(i).max_rep == 0]
    for col in flat:
        path = f.column_info(col).path.decode()
        exp = pqtest.pyarrow_flat(data, path)
        for rg in range(f.num_row_groups):
            cd = f.read_chunk(rg, col)
            vals, valid = exp[rg]
            np.testing.assert_array_equal(cd.def_levels == f.column_info(col).max_def, valid)
            if vals is None:
                continue
            got = pqtest.oracle_values(cd)
            if isinstance(vals, list):
                assert got == vals
            else:
                assert np.asarray(got).tobytes() == np.asarray(vals).tobytes(), (name, path, rg)
    assert pf.metadata.num_row_groups == f.num_row_groups


def test_oracle_nested_levels():
    """LIST<INT32> / MAP levels derived from pyarrow's nested arrays (Dremel encoding)."""
    import io
    import pyarrow.parquet as pq
    data = pqtest.load("cfg4_small")
    t = pq.read_table(io.BytesIO(data))
    f = O.File(data)
    lists = t.column("l").combine_chunks().to_pylist()
    # expected levels for l.list.element: maxD 3 (list optional, repeated, element optional), maxR 1
    dl, rl, vals = [], [], []
    for rec in lists:
        if rec is None:
            dl.append(0); rl.append(0)
        elif len(rec) == 0:
            dl.append(1); rl.append(0)
        else:
            for i, e in enumerate(rec):
                rl.append(0 if i == 0 else 1)
                dl.append(2 if e is None else 3)
                if e is not None:
                    vals.append(e)
    got_dl, got_rl, got_v = [], [], []
    for rg in range(f.num_row_groups):
        cd = f.read_chunk(rg, 0)
        got_dl += list(cd.def_levels)
        got_rl += list(cd.rep_levels)
        got_v += list(cd.values)
    assert got_dl == dl and got_rl == rl and got_v == vals


@pytest.mark.parametrize("name,expected", sorted(pqtest.EXPECTED_ERRORS.items()))
def test_oracle_expected_errors(name, expected):
    code, page = expected
    errs = [r for _, _, r in pqtest.oracle_decode(pqtest.load(name)) if isinstance(r, O.OracleError)]
    assert errs, name
    assert (errs[0].code, errs[0].page) == (code, page), (name, errs[0])


def test_must_not_crash_oracle():
    """The reference's fuzz regression images (fuzz_test.go etc.): decode must return, not crash."""
    d = os.path.join(pqtest.GOLDEN, "must_not_crash")
    n = 0
    for fn in sorted(os.listdir(d)):
        data = open(os.path.join(d, fn), "rb").read()
        try:
            f = O.File(data)
        except O.OracleError:
            n += 1
            continue
        for rg in range(f.num_row_groups):
            for col in range(f.num_columns):
                try:
                    f.read_chunk(rg, col)
                except O.OracleError:
                    pass
        n += 1
    assert n >= 8
