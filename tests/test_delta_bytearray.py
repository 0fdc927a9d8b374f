"""DELTA_LENGTH_BYTE_ARRAY and DELTA_BYTE_ARRAY (type_bytearray.go:98-240; SURVEY.md §8(a)
a13, §8(f) rank 1). Streams are built from the format specification by tools/rawpq.py:
valid pages of both encodings over several lengths-stream shapes (128/4 as the reference
writer, 256/8, miniblocks of 4 values which take the exact scalar path), the look-ahead
quirk (App. A Q1: N = 1 mod block size fails in init), negative lengths, truncated
payloads, prefixes longer than the previous value, negative prefixes and prefix/suffix
count mismatches. The oracle must return the generator's values (or the reference's
error class); the GPU must equal the oracle."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import rawpq  # noqa: E402

import pqtest  # noqa: E402
import py_oracle as O  # noqa: E402


def _words(rng, n, shared=0.0):
    """n byte strings; with `shared`, runs of values share growing prefixes (sorted-key style)."""
    out, prev = [], b""
    for _ in range(n):
        if prev and rng.random() < shared:
            k = int(rng.integers(0, len(prev) + 1))
            v = prev[:k] + bytes(rng.integers(97, 123, int(rng.integers(0, 12)), dtype=np.uint8))
        else:
            v = bytes(rng.integers(97, 123, int(rng.integers(0, 24)), dtype=np.uint8))
        out.append(v)
        prev = v
    return out


SHAPES = [(128, 4), (256, 8), (128, 1), (128, 32), (4096, 512)]  # (block size, miniblocks); 128/32: 4-value miniblocks
COUNTS = [2, 7, 8, 100, 128, 130, 1000, 4000]  # 1: no block at all, see dlba_single


def _valid_file(k, enc, v2):
    bs, mbc = SHAPES[k]
    rng = np.random.default_rng(40 + k)
    pages, expect = [], []
    for c in COUNTS:
        if c > 1 and c % bs == 1:
            continue
        vals = _words(rng, c, shared=0.7 if enc == "DELTA_BYTE_ARRAY" else 0.0)
        if enc == "DELTA_LENGTH_BYTE_ARRAY":
            st = rawpq.dlba_stream([len(v) for v in vals], b"".join(vals), bs, mbc)
        else:
            st = rawpq.dba_stream(*rawpq.dba_encode(vals), bs, mbc)
        pages.append((st, c))
        expect += vals
    return rawpq.ba_column_file(pages, enc, v2), expect


def _oracle_values(data):
    r = O.File(data).read_chunk(0, 0)
    return pqtest.oracle_values(r)


CASES = [(k, enc, v2) for k in range(len(SHAPES)) for enc in ("DELTA_LENGTH_BYTE_ARRAY", "DELTA_BYTE_ARRAY")
         for v2 in (False, True)]


@pytest.mark.parametrize("k,enc,v2", CASES)
def test_oracle_valid(k, enc, v2):
    bs, mbc = SHAPES[k]
    if (bs // mbc) % 8:
        pytest.skip("miniblocks of 4 values: the reference reads 8 at a time across them (GPU test compares)")
    data, expect = _valid_file(k, enc, v2)
    assert _oracle_values(data) == expect


def _bad_files():
    """name -> (file bytes, expected oracle error class or None)."""
    rng = np.random.default_rng(7)
    vals = _words(rng, 300)
    lens = [len(v) for v in vals]
    pay = b"".join(vals)
    out = {}
    # Q1: 129 lengths in 128-value blocks: init reads the 2nd block header from the payload
    # bytes (here: a miniblock width > 32 -> invalid)
    # a single value: the writer emits no block, so init() reads its miniblock header from the
    # payload (whatever the reference makes of that, the GPU must make of it too)
    out["dlba_single"] = (rawpq.ba_column_file([(rawpq.dlba_stream(lens[:1], vals[0]), 1)], "DELTA_LENGTH_BYTE_ARRAY"),
                          "any")
    out["dlba_q1"] = (rawpq.ba_column_file([(rawpq.dlba_stream(lens[:129], b"".join(vals[:129])), 129)],
                                           "DELTA_LENGTH_BYTE_ARRAY"), 3)
    bad = list(lens)
    bad[77] = -3
    out["dlba_negative_len"] = (rawpq.ba_column_file([(rawpq.dlba_stream(bad, pay), 300)], "DELTA_LENGTH_BYTE_ARRAY"), 3)
    out["dlba_short_payload"] = (rawpq.ba_column_file([(rawpq.dlba_stream(lens, pay[:-5]), 300)],
                                                      "DELTA_LENGTH_BYTE_ARRAY"), 2)
    cut = sum(lens[:200])
    out["dlba_payload_at_eof"] = (rawpq.ba_column_file([(rawpq.dlba_stream(lens[:200] + [5] * 100, pay[:cut]), 300)],
                                                       "DELTA_LENGTH_BYTE_ARRAY"), 1)
    svals = _words(rng, 300, shared=0.8)
    pre, sl, spay = rawpq.dba_encode(svals)
    p2 = list(pre)
    p2[150] = len(svals[149]) + 2
    out["dba_prefix_too_long"] = (rawpq.ba_column_file([(rawpq.dba_stream(p2, sl, spay), 300)], "DELTA_BYTE_ARRAY"), 3)
    p3, s3 = list(pre), list(sl)
    p3[60], s3[60] = -2, 5  # negative prefix, long enough suffix: the value is the suffix alone
    spay3 = b"".join(svals[i][pre[i]:] if i != 60 else b"zzzzz" for i in range(300))
    out["dba_negative_prefix"] = (rawpq.ba_column_file([(rawpq.dba_stream(p3, s3, spay3), 300)], "DELTA_BYTE_ARRAY"),
                                  None)
    p4, s4 = list(pre), list(sl)
    p4[61], s4[61] = -9, 2  # prefix + suffix < 0: Go's make() panics
    spay4 = b"".join(svals[i][pre[i]:] if i != 61 else b"zz" for i in range(300))
    out["dba_negative_cap"] = (rawpq.ba_column_file([(rawpq.dba_stream(p4, s4, spay4), 300)], "DELTA_BYTE_ARRAY"), 3)
    out["dba_count_mismatch"] = (rawpq.ba_column_file([(rawpq.dba_stream(pre[:299], sl, spay), 300)],
                                                      "DELTA_BYTE_ARRAY"), 3)
    out["dba_more_values_than_lengths"] = (rawpq.ba_column_file([(rawpq.dba_stream(pre[:250], sl[:250], spay), 300)],
                                                                "DELTA_BYTE_ARRAY"), 1)
    return out


BAD = _bad_files()


@pytest.mark.parametrize("name", sorted(BAD))
def test_oracle_errors(name):
    data, code = BAD[name]
    f = O.File(data)
    if code == "any":
        return
    if code is None:
        f.read_chunk(0, 0)
    else:
        with pytest.raises(O.OracleError) as ei:
            f.read_chunk(0, 0)
        assert ei.value.code == code, (name, ei.value)


def _gpu(ctx, data):
    import pqgpu
    f = pqgpu.File(data)
    b = pqgpu.Batch(ctx)
    cid, e = b.add_file_chunk(f, 0, 0)
    b.decode()
    b.sync()
    out = e or b.status(cid) or b.result(cid)
    b.close()
    return out


def _compare(gpu, data, where):
    import pqgpu
    try:
        orc = O.File(data).read_chunk(0, 0)
    except O.OracleError as r:
        assert isinstance(gpu, pqgpu.DecodeError), f"{where}: oracle error {r} but GPU decoded"
        assert (gpu.code, gpu.page) == (r.code, r.page), f"{where}: {gpu} vs {r}"
        return
    assert not isinstance(gpu, pqgpu.DecodeError), f"{where}: GPU error {gpu}"
    pqtest.assert_chunk_equal(gpu, orc, where)


@pytest.mark.gpu
@pytest.mark.parametrize("k,enc,v2", CASES)
def test_gpu_valid(gpu_ctx, k, enc, v2):
    data, _ = _valid_file(k, enc, v2)
    _compare(_gpu(gpu_ctx, data), data, f"{SHAPES[k]} {enc} v2={v2}")


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(BAD))
def test_gpu_errors(gpu_ctx, name):
    data, _ = BAD[name]
    _compare(_gpu(gpu_ctx, data), data, name)


# ---------------------------------------------------------------- FIXED_LEN_BYTE_ARRAY x DELTA_BYTE_ARRAY
# getFixedLenByteArrayValuesDecoder (chunk_reader.go:64-75) returns byteArrayDeltaDecoder for
# DELTA_BYTE_ARRAY pages: values of any length (the type length is not checked), so the GPU lays
# such a chunk out as byte arrays; its PLAIN pages (byteArrayPlainDecoder{length}) and dictionary
# entries are type_length bytes each.

def _flba_file(v2=False, with_dict=False):
    rng = np.random.default_rng(91)
    tl = 12
    fixed = [bytes(rng.integers(0, 256, tl, dtype=np.uint8)) for _ in range(500)]
    fixed.sort()
    ragged = _words(rng, 300, shared=0.6)  # the reference accepts other lengths on DBA pages
    pages, expect = [], []
    if with_dict:
        dvals = fixed[:40]
        pages.append(rawpq.dict_page_ref("FIXED_LEN_BYTE_ARRAY", dvals, tl))
        idx = rng.integers(0, 40, 700)
        body = rawpq.dict_values_section(idx, 40)
        pages.append(rawpq.data_page_v2_ref(700, 0, 700, "RLE_DICTIONARY", body) if v2
                     else rawpq.data_page_v1_ref(700, "RLE_DICTIONARY", body))
        expect += [dvals[i] for i in idx]
    for vals, enc in ((fixed[:250], "DELTA_BYTE_ARRAY"), (fixed[250:], "PLAIN"), (ragged, "DELTA_BYTE_ARRAY")):
        body = rawpq.dba_stream(*rawpq.dba_encode(vals)) if enc == "DELTA_BYTE_ARRAY" else \
            rawpq.plain_encode("FIXED_LEN_BYTE_ARRAY", vals, tl)
        n = len(vals)
        pages.append(rawpq.data_page_v2_ref(n, 0, n, enc, body) if v2 else rawpq.data_page_v1_ref(n, enc, body))
        expect += vals
    schema = [[(4, rawpq.BIN, "schema"), (5, rawpq.I32, 1)], rawpq.schema_leaf("f", "FIXED_LEN_BYTE_ARRAY", "REQUIRED", tl)]
    n = len(expect)
    return rawpq.write_file_schema(schema, [("f", "FIXED_LEN_BYTE_ARRAY")], [(n, [(pages, n, with_dict)])]), expect


FLBA_CASES = [(v2, d) for v2 in (False, True) for d in (False, True)]


@pytest.mark.parametrize("v2,with_dict", FLBA_CASES)
def test_oracle_flba_dba(v2, with_dict):
    data, expect = _flba_file(v2, with_dict)
    assert _oracle_values(data) == expect


def test_host_plans_flba_dba():
    import pqgpu
    data, _ = _flba_file()
    b = pqgpu.Batch(None)
    cid, e = b.add_file_chunk(pqgpu.File(data), 0, 0)
    assert e is None, e
    b.close()


@pytest.mark.gpu
@pytest.mark.parametrize("v2,with_dict", FLBA_CASES)
def test_gpu_flba_dba(gpu_ctx, v2, with_dict):
    data, expect = _flba_file(v2, with_dict)
    g = _gpu(gpu_ctx, data)
    _compare(g, data, f"flba dba v2={v2} dict={with_dict}")
    assert g.values == expect
