"""Generate the small Parquet fixtures under tests/golden/ (pyarrow writer).

The files are the BASELINE.json config shapes scaled down to a few hundred KB
each, plus edge cases (all-null pages, single values, every physical type,
codecs, V1/V2 pages) and deliberately corrupted variants (see corrupt()).
Expected outputs are NOT stored here: tests decode each file with the CPU
oracle (oracle/, pinned by the reference's own known-answer tests) and with
pyarrow, and compare the GPU decoder against both.

Seeds follow SURVEY.md §8(d) (numpy default_rng). Re-running this script
rewrites the same bytes for a given pyarrow version (25.0.0 here).

    python tools/gen_fixtures.py            # writes tests/golden/*.parquet
"""
import io
import json
import os
import sys

import numpy as np
import pyarrow as pa
import pyarrow.parquet as pq

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(os.path.dirname(HERE), "tests", "golden")
sys.path.insert(0, HERE)
import pqinspect  # noqa: E402


def write(table, **kw):
    b = io.BytesIO()
    pq.write_table(table, b, **kw)
    return b.getvalue()


def delta_safe(mask, page_rows, block=256):
    """True if no page's non-null count is ≡ 1 (mod block)."""
    nn = (~mask).astype(np.int64)
    for s in range(0, len(nn), page_rows):
        c = int(nn[s:s + page_rows].sum())
        if c % block == 1 or c == 1 or c == 0:
            return False
    return True


def cfg1(n=100_000, page_rows=16384):
    # INT32 REQUIRED, 255-entry dictionary (bw=8), V1, UNCOMPRESSED (seed 1)
    rng = np.random.default_rng(1)
    d = rng.integers(-2**31, 2**31 - 1, 255, dtype=np.int64).astype(np.int32)
    idx = rng.integers(0, 255, n)
    t = pa.table({"a": pa.array(d[idx], pa.int32())}, schema=pa.schema([pa.field("a", pa.int32(), nullable=False)]))
    return write(t, use_dictionary=True, data_page_version="1.0", compression="NONE", max_rows_per_page=page_rows)


def cfg2(n=150_000, page_rows=16384, rg=75_000, version="2.0", compression="NONE", seed=2):
    # INT64 DELTA_BINARY_PACKED + DOUBLE PLAIN, OPTIONAL 10% nulls (seeds 2, 3)
    rng = np.random.default_rng(seed)
    while True:
        a = np.cumsum(rng.integers(0, 2**16, n)).astype(np.int64)
        m = rng.random(n) < 0.1
        if all(delta_safe(m[s:s + rg], page_rows) for s in range(0, n, rg)):
            break
    rng3 = np.random.default_rng(seed + 1)
    b = rng3.random(n)
    m2 = rng3.random(n) < 0.1
    t = pa.table({"a": pa.array(a, mask=m), "b": pa.array(b, mask=m2)})
    return write(t, use_dictionary=False, data_page_version=version, compression=compression,
                 column_encoding={"a": "DELTA_BINARY_PACKED", "b": "PLAIN"}, max_rows_per_page=page_rows,
                 row_group_size=rg)


def words(rng, k, lo=4, hi=28):
    out = set()
    while len(out) < k:
        ln = int(rng.integers(lo, hi + 1))
        out.add(bytes(rng.integers(97, 123, ln, dtype=np.uint8)).decode())
    return sorted(out)


def cfg3(n=120_000, k=4096, page_rows=None):
    # BYTE_ARRAY REQUIRED, dictionary of k strings (bw=12 at 4096), V1 (seed 4)
    rng = np.random.default_rng(4)
    vocab = np.array(words(rng, k), dtype=object)
    s = vocab[rng.integers(0, k, n)]
    t = pa.table({"s": pa.array(list(s), pa.string())}, schema=pa.schema([pa.field("s", pa.string(), nullable=False)]))
    kw = dict(use_dictionary=True, data_page_version="1.0", compression="NONE", dictionary_pagesize_limit=8 << 20)
    if page_rows:
        kw["max_rows_per_page"] = page_rows
    return write(t, **kw)


def cfg1_full():
    # cfg1 exactly as BASELINE.json configs[0] / SURVEY §8(d): 1,048,576 rows, 8 pages of 131,072
    return cfg1(1_048_576, 131_072)


def cfg3_dict64k(n=262_144, k=65_536, page_rows=65_536):
    # cfg3's defining shape: a 65,536-entry BYTE_ARRAY dictionary (lengths 4-28, mean 16) with
    # 16-bit indices. The first k rows are a permutation of the vocabulary, so every entry is
    # used and pyarrow's index width is bit_width(k - 1) = 16 (seed 4).
    rng = np.random.default_rng(4)
    vocab = np.array(words(rng, k), dtype=object)
    idx = np.concatenate([rng.permutation(k), rng.integers(0, k, n - k)])
    t = pa.table({"s": pa.array(list(vocab[idx]), pa.string())},
                 schema=pa.schema([pa.field("s", pa.string(), nullable=False)]))
    return write(t, use_dictionary=True, data_page_version="1.0", compression="NONE",
                 dictionary_pagesize_limit=8 << 20, max_rows_per_page=page_rows)


def crc_files():
    """Page checksums (pyarrow write_page_checksum; checked with WithCRC32Validation,
    file_reader.go:134-139, chunk_reader.go:173-177): a valid file, and the same file with one
    value byte of the second data page of column `a` flipped (still decodable without the
    check; CRC32 check failed on that page with it)."""
    rng = np.random.default_rng(31)
    n = 20_000
    t = pa.table({"a": pa.array(rng.integers(0, 1 << 40, n, dtype=np.int64), mask=rng.random(n) < 0.1),
                  "s": pa.array(["v%d" % (i % 37) for i in range(n)])})
    good = write(t, data_page_version="1.0", compression="NONE", use_dictionary=["s"], max_rows_per_page=4096,
                 write_page_checksum=True)
    buf = bytearray(good)
    ph, j = [(ph, j) for ph, j in pqinspect.pages(good) if ph[1] == 0][1]
    csize = ph[3]
    buf[j + csize - 5] ^= 0x5A  # a PLAIN value byte near the end of the page
    return {"crc_v1": good, "crc_v1_flipped": bytes(buf)}


def cfg4(n=20_000, version="1.0", seed=5):
    # LIST<INT32> + MAP<BYTE_ARRAY, INT64> (seed 5)
    rng = np.random.default_rng(seed)
    vocab = words(rng, 1024, 3, 10)
    lists, maps = [], []
    for _ in range(n):
        u = rng.random()
        if u < 0.05:
            lists.append(None)
        elif u < 0.10:
            lists.append([])
        else:
            ln = int(rng.integers(1, 9))
            el = rng.integers(-2**31, 2**31 - 1, ln).tolist()
            nulls = rng.random(ln) < 0.05
            lists.append([None if z else int(e) for e, z in zip(el, nulls)])
        if rng.random() < 0.05:
            maps.append(None)
        else:
            ln = int(rng.integers(0, 5))
            keys = rng.choice(len(vocab), ln, replace=False)
            vals = rng.integers(-2**62, 2**62, ln)
            vn = rng.random(ln) < 0.05
            maps.append([(vocab[int(kk)], None if z else int(v)) for kk, v, z in zip(keys, vals, vn)])
    t = pa.table({"l": pa.array(lists, pa.list_(pa.int32())), "m": pa.array(maps, pa.map_(pa.string(), pa.int64()))})
    return write(t, data_page_version=version, compression="NONE", use_dictionary=["m.key_value.key"],
                 max_rows_per_page=4096)


def struct_files(n=20_000, seed=7):
    """OPTIONAL groups (structs) at list depth 0 and 1, around and inside lists, plus a MAP (f3:
    struct validity and shared map offsets; Column.getNextData schema.go:216-260):
      s  : struct<a: int32, l: list<int32>>, 5 % null structs, a 10 % null, l 5 % null / 5 % empty
      ls : list<struct<x: int32, y: string>>, 5 % null lists, 5 % null struct elements
      t  : struct<u: struct<x: int64 (required)>>, 5 % null t, 5 % null u
      mm : map<string, int32>, 5 % null maps, 0-3 entries, 10 % null values"""
    rng = np.random.default_rng(seed)

    def i32():
        return int(rng.integers(-2**31, 2**31 - 1))

    s, ls, t, mm = [], [], [], []
    for _ in range(n):
        if rng.random() < 0.05:
            s.append(None)
        else:
            u = rng.random()
            lst = None if u < 0.05 else [] if u < 0.10 else [
                None if rng.random() < 0.05 else i32() for _ in range(int(rng.integers(1, 5)))]
            s.append({"a": None if rng.random() < 0.10 else i32(), "l": lst})
        if rng.random() < 0.05:
            ls.append(None)
        else:
            ls.append([None if rng.random() < 0.05 else
                       {"x": None if rng.random() < 0.10 else i32(), "y": "w%d" % int(rng.integers(0, 50))}
                       for _ in range(int(rng.integers(0, 4)))])
        u = rng.random()
        t.append(None if u < 0.05 else {"u": None} if u < 0.10 else {"u": {"x": int(rng.integers(-2**62, 2**62))}})
        if rng.random() < 0.05:
            mm.append(None)
        else:
            ks = rng.choice(40, int(rng.integers(0, 4)), replace=False)
            mm.append([("k%d" % int(k), None if rng.random() < 0.10 else i32()) for k in ks])
    tbl = pa.table({
        "s": pa.array(s, pa.struct([("a", pa.int32()), ("l", pa.list_(pa.int32()))])),
        "ls": pa.array(ls, pa.list_(pa.struct([("x", pa.int32()), ("y", pa.string())]))),
        "t": pa.array(t, pa.struct([("u", pa.struct([pa.field("x", pa.int64(), nullable=False)]))])),
        "mm": pa.array(mm, pa.map_(pa.string(), pa.int32())),
    })
    return {"struct_v1": write(tbl, data_page_version="1.0", compression="NONE", max_rows_per_page=4096),
            "struct_v2": write(tbl, data_page_version="2.0", compression="NONE", max_rows_per_page=4096)}


def cfg5(n=60_000, rg=20_000, compression="SNAPPY"):
    # 8-column mix (INT32 dict / INT64 DELTA / DOUBLE PLAIN / INT64 PLAIN), REQUIRED, V1
    rng = np.random.default_rng(6)
    cols, enc = {}, {}
    fields = []
    for i in range(2):
        d = rng.integers(-2**31, 2**31 - 1, 200, dtype=np.int64).astype(np.int32)
        cols[f"d{i}"] = pa.array(d[rng.integers(0, 200, n)], pa.int32())
        cols[f"e{i}"] = pa.array(np.cumsum(rng.integers(-1000, 1000, n)).astype(np.int64))
        enc[f"e{i}"] = "DELTA_BINARY_PACKED"
        cols[f"f{i}"] = pa.array(rng.random(n))
        enc[f"f{i}"] = "PLAIN"
        cols[f"g{i}"] = pa.array(rng.integers(-2**63, 2**63 - 1, n, dtype=np.int64))
        enc[f"g{i}"] = "PLAIN"
    for k, v in cols.items():
        fields.append(pa.field(k, v.type, nullable=False))
    t = pa.table(cols, schema=pa.schema(fields))
    return write(t, compression=compression, data_page_version="1.0", row_group_size=rg,
                 use_dictionary=[k for k in cols if k.startswith("d")], column_encoding=enc, max_rows_per_page=8192)


def types_v(version):
    # every physical type, OPTIONAL, both page versions
    import datetime
    rng = np.random.default_rng(7)
    n = 5000
    mk = lambda: rng.random(n) < 0.2  # noqa: E731
    ts = [datetime.datetime(2001, 1, 1) + datetime.timedelta(microseconds=int(x)) for x in rng.integers(0, 10**14, n)]
    f32 = rng.standard_normal(n).astype(np.float32)
    f32[::97] = np.float32("nan")
    f64 = rng.standard_normal(n)
    f64[::89] = np.nan
    t = pa.table({
        "bool": pa.array(rng.random(n) < 0.3, mask=mk()),
        "i32": pa.array(rng.integers(-2**31, 2**31 - 1, n, dtype=np.int64).astype(np.int32), mask=mk()),
        "i64": pa.array(rng.integers(-2**63, 2**63 - 1, n, dtype=np.int64), mask=mk()),
        "i96": pa.array(ts, pa.timestamp("us"), mask=mk()),
        "f32": pa.array(f32, mask=mk()),
        "f64": pa.array(f64, mask=mk()),
        "str": pa.array([bytes(rng.integers(0, 256, int(rng.integers(0, 40)), dtype=np.uint8)) for _ in range(n)],
                        pa.binary(), mask=mk()),
        "flba": pa.array([bytes(rng.integers(0, 256, 12, dtype=np.uint8)) for _ in range(n)], pa.binary(12),
                         mask=mk()),
    })
    return write(t, data_page_version=version, compression="NONE", use_dictionary=False,
                 use_deprecated_int96_timestamps=True, max_rows_per_page=1500)


def types_dict():
    rng = np.random.default_rng(8)
    n = 6000
    t = pa.table({
        "i64": pa.array(rng.integers(0, 50, n).astype(np.int64) * 1234567890123),
        "f64": pa.array(rng.integers(0, 30, n).astype(np.float64) / 7),
        "f32": pa.array((rng.integers(0, 30, n) / 3).astype(np.float32)),
        "flba": pa.array([bytes([i % 7] * 6) for i in rng.integers(0, 40, n)], pa.binary(6)),
        "str": pa.array(["k%03d" % i for i in rng.integers(0, 300, n)], mask=rng.random(n) < 0.1),
        "one": pa.array(np.full(n, 42, np.int32)),  # single-entry dictionary: bit width 0
    })
    return write(t, data_page_version="1.0", compression="NONE", use_dictionary=True, max_rows_per_page=2000)


def edge_cases():
    rng = np.random.default_rng(9)
    files = {}
    # all-null pages, long RLE runs, empty row group at the end
    n = 40_000
    m = np.zeros(n, bool)
    m[5000:25000] = True
    files["edge_nulls_v1"] = write(pa.table({"a": pa.array(np.arange(n, dtype=np.int64), mask=m),
                                             "z": pa.array([None] * n, pa.int32())}),
                                   data_page_version="1.0", compression="NONE", use_dictionary=False,
                                   max_rows_per_page=4096)
    files["edge_nulls_v2"] = write(pa.table({"a": pa.array(np.arange(n, dtype=np.int64), mask=m)}),
                                   data_page_version="2.0", compression="NONE", use_dictionary=False,
                                   max_rows_per_page=4096)
    # tiny pages (1-3 values), many pages
    files["edge_tiny_pages"] = write(pa.table({"a": pa.array(rng.integers(0, 9, 300).astype(np.int32)),
                                               "s": pa.array(["x" * int(i) for i in rng.integers(0, 5, 300)])}),
                                     data_page_version="1.0", compression="NONE", max_rows_per_page=3)
    # DELTA INT32 with wrapping arithmetic and huge deltas; 32-bit widths
    v = rng.integers(-2**31, 2**31 - 1, 20_000, dtype=np.int64).astype(np.int32)
    files["edge_delta32"] = write(pa.table({"a": pa.array(v)}), use_dictionary=False, compression="NONE",
                                  column_encoding={"a": "DELTA_BINARY_PACKED"}, max_rows_per_page=5000)
    # DELTA INT64 with 64-bit widths
    v = rng.integers(-2**63, 2**63 - 1, 20_000, dtype=np.int64)
    files["edge_delta64_wide"] = write(pa.table({"a": pa.array(v)}), use_dictionary=False, compression="NONE",
                                       column_encoding={"a": "DELTA_BINARY_PACKED"}, max_rows_per_page=7000)
    # Q1: a DELTA page with N ≡ 1 (mod 256) non-null values -> the reference fails with EOF
    files["edge_delta_q1"] = write(pa.table({"a": pa.array(np.arange(257, dtype=np.int64))}), use_dictionary=False,
                                   compression="NONE", column_encoding={"a": "DELTA_BINARY_PACKED"})
    # GZIP V2 and SNAPPY V1 with levels
    files["cfg2_gzip_v2"] = cfg2(40_000, 8192, 20_000, "2.0", "GZIP", seed=12)
    files["cfg2_snappy_v1"] = cfg2(40_000, 8192, 40_000, "1.0", "SNAPPY", seed=14)
    # nested V2
    files["cfg4_v2"] = cfg4(6000, "2.0", seed=15)
    # empty table
    files["edge_empty"] = write(pa.table({"a": pa.array([], pa.int64())}), compression="NONE")
    return files


def delta_ba():
    """DELTA_LENGTH_BYTE_ARRAY / DELTA_BYTE_ARRAY columns as pyarrow writes them (lengths in
    128-value blocks). Page non-null counts avoid N = 1 (mod 128) (App. A Q1)."""
    rng = np.random.default_rng(21)
    n = 12_000
    w = words(rng, 2000)
    keys = sorted(f"user/{int(i):08d}/" + w[int(i) % len(w)] for i in rng.integers(0, 10**7, n))
    vals = [w[int(i)] for i in rng.integers(0, len(w), n)]
    m = rng.random(n) < 0.1
    page_rows = 3000
    pages = m.reshape(-1, page_rows)
    for p in np.flatnonzero((page_rows - pages.sum(1)) % 128 == 1):
        pages[p, np.flatnonzero(pages[p])[0]] = False
    files = {}
    t = pa.table({"s": pa.array(vals, mask=m), "k": pa.array(keys)})
    files["dlba_v1"] = write(t, use_dictionary=False, data_page_version="1.0", compression="NONE",
                             column_encoding={"s": "DELTA_LENGTH_BYTE_ARRAY", "k": "DELTA_LENGTH_BYTE_ARRAY"},
                             max_rows_per_page=page_rows)
    files["dba_v2"] = write(t, use_dictionary=False, data_page_version="2.0", compression="NONE",
                            column_encoding={"s": "DELTA_BYTE_ARRAY", "k": "DELTA_BYTE_ARRAY"},
                            max_rows_per_page=page_rows)
    files["dba_v1_snappy"] = write(t, use_dictionary=False, data_page_version="1.0", compression="SNAPPY",
                                   column_encoding={"s": "DELTA_BYTE_ARRAY", "k": "DELTA_LENGTH_BYTE_ARRAY"},
                                   max_rows_per_page=page_rows)
    return files


def pqinspect_uvar_bytes(x):
    out = bytearray()
    while True:
        if x < 0x80:
            out.append(x)
            return bytes(out)
        out.append((x & 0x7F) | 0x80)
        x >>= 7


def corrupt(files):
    """Byte-patched variants with known reference error classes."""
    out = {}
    # dictionary index out of range: shrink the dictionary header's num_values
    buf = bytearray(files["cfg1"])
    # first data page of cfg1: the index stream starts after the bit-width byte; set one index to 255 (bw 8 -> fits
    # 8 bits but dictionary has 255 entries, so 255 is out of range)
    it = list(pqinspect.pages(bytes(buf)))
    dp = [(ph, j) for ph, j in it if ph[1] == 0][1]
    ph, j = dp
    # V1 REQUIRED: values section starts at j; byte 0 = bit width; then run header(s)
    bw = buf[j]
    assert bw == 8
    h, k = pqinspect.uvar(buf, j + 1)
    assert h & 1
    buf[k + 100] = 255
    out["bad_dict_index"] = bytes(buf)
    # truncated DELTA stream: page header says more bytes than the chunk has -> short block read
    b2 = bytearray(files["edge_delta32"])
    it = list(pqinspect.pages(bytes(b2)))
    ph, j = it[1]
    # corrupt a miniblock bit width to 40 (> 32) in the page's first block header
    # layout: blockSize, mbc, count, first, minDelta, widths...
    p = j
    for _ in range(4):
        _, p = pqinspect.uvar(b2, p)
    _, p = pqinspect.uvar(b2, p)  # min delta
    b2[p] = 40
    out["bad_delta_width"] = bytes(b2)
    # hybrid def levels: zero-count RLE run inside a V2 def section
    b4 = bytearray(files["cfg2_v2_small"])
    ph, j = [(ph, j) for ph, j in pqinspect.pages(bytes(b4)) if ph[1] == 3][2]
    dl, rl = ph[8][5], ph[8][6]
    # overwrite the 3rd run header with 0x00 (RLE, count 0)
    runs = []
    q = j + rl
    end = q + dl
    while q < end and len(runs) < 3:
        h, q2 = pqinspect.uvar(b4, q)
        runs.append(q)
        q = q2 + ((h >> 1) * 1 if h & 1 else 1)
    b4[runs[2]] = 0
    out["bad_def_empty_run"] = bytes(b4)
    # V2 page header whose num_nulls disagrees with its definition levels: the reference
    # ignores the field (notNull is counted from the levels, page_v2.go:47-50), so the file
    # decodes; the GPU decoder's speculative value bases miss and it re-runs serially.
    b5 = bytearray(files["cfg2_v2_small"])
    ph, j = [(ph, j) for ph, j in pqinspect.pages(bytes(b5)) if ph[1] == 3][1]
    nv, nulls = ph[8][1], ph[8][2]
    zz = lambda v: pqinspect_uvar_bytes((v << 1) ^ (v >> 31))
    pat = b"\x15" + zz(nv) + b"\x15" + zz(nulls)
    k = bytes(b5).rfind(pat, 0, j)
    assert k > 0
    new = zz(nulls + 1) if len(zz(nulls + 1)) == len(zz(nulls)) else zz(nulls - 1)
    q = k + 2 + len(zz(nv))
    b5[q:q + len(new)] = new
    out["bad_v2_num_nulls"] = bytes(b5)
    # truncated file: cut the last data page of cfg2_v2_small in half (chunk-level read error)
    out["truncated"] = files["cfg1"][: len(files["cfg1"]) // 2] + files["cfg1"][-(8 + 400):]
    return out


def main():
    os.makedirs(OUT, exist_ok=True)
    if len(sys.argv) > 1 and sys.argv[1] == "--only-struct":  # add the f3 fixtures alone
        for name, data in struct_files().items():
            with open(os.path.join(OUT, name + ".parquet"), "wb") as f:
                f.write(data)
        return
    files = {
        "cfg1": cfg1(),
        "cfg2_v2_small": cfg2(),
        "cfg3_small": cfg3(),
        "cfg4_small": cfg4(),
        "cfg5_small": cfg5(),
        "types_v1": types_v("1.0"),
        "types_v2": types_v("2.0"),
        "types_dict": types_dict(),
    }
    files["cfg1_full"] = cfg1_full()
    files["cfg3_dict64k"] = cfg3_dict64k()
    files.update(crc_files())
    files.update(edge_cases())
    files.update(delta_ba())
    files.update(struct_files())
    files.update(corrupt(files))
    manifest = {}
    for name, data in sorted(files.items()):
        with open(os.path.join(OUT, name + ".parquet"), "wb") as f:
            f.write(data)
        manifest[name] = {"bytes": len(data)}
    with open(os.path.join(OUT, "fixtures.json"), "w") as f:
        json.dump({"pyarrow": pa.__version__, "files": manifest}, f, indent=1, sort_keys=True)
    print(f"wrote {len(files)} fixtures, {sum(len(v) for v in files.values()) / 1e6:.2f} MB")


if __name__ == "__main__":
    main()
