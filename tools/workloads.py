"""Synthetic BASELINE.json workloads for bench.py (benchmark infrastructure, not product code).

Every generator follows SURVEY.md §8(d) (shapes, seeds from numpy default_rng) and returns
(file bytes, truth) where `truth` holds what a verifier needs (None when not kept). Files are
written by pyarrow 25 (present in this image and on the GPU box); generators build Arrow arrays
from numpy buffers so that the largest (cfg4, 16 Mi records) takes seconds, not minutes.

  cfg1  INT32 REQUIRED, 255-entry dictionary (bw 8), V1, 1,048,576 rows in 8 pages of 131,072
  cfg2  INT64 DELTA + DOUBLE PLAIN, OPTIONAL 10 % nulls, V2, 67,108,864 rows, 16 row groups
  cfg3  BYTE_ARRAY REQUIRED, 65,536-entry dictionary (lengths 4-28), 16-bit indices, V1,
        33,554,432 rows, 8 row groups of 4,194,304 (one dictionary per row group)
  cfg4  LIST<INT32> + MAP<BYTE_ARRAY, INT64>, 16,777,216 records, V1, 4 row groups
  cfg5  64 REQUIRED columns (16 each: INT32 dictionary bw 8, INT64 DELTA, DOUBLE PLAIN, INT64
        PLAIN), SNAPPY, V1, row groups of 3,906,250 rows: a few row-group templates written by
        pyarrow, their bytes replicated behind a rewritten footer
"""
import io

import numpy as np

RG_ROWS = 4_194_304


def _write(table, **kw):
    import pyarrow.parquet as pq
    bio = io.BytesIO()
    pq.write_table(table, bio, write_statistics=False, **kw)
    return bio.getvalue()


def gen_cfg1(rows=1_048_576, page_rows=131_072, seed=1, first_rg=0):
    """cfg1 (configs[0]): the reference's CPU-runnable case."""
    import pyarrow as pa
    rng = np.random.default_rng(seed)
    d = rng.integers(-2**31, 2**31 - 1, 255, dtype=np.int64).astype(np.int32)
    idx = rng.integers(0, 255, rows)
    vals = d[idx]
    t = pa.table({"a": pa.array(vals, pa.int32())}, schema=pa.schema([pa.field("a", pa.int32(), nullable=False)]))
    return _write(t, use_dictionary=True, data_page_version="1.0", compression="NONE", max_rows_per_page=page_rows,
                  row_group_size=max(rows, 1)), vals


def gen_cfg2(rows=67_108_864, rg_rows=RG_ROWS, page_rows=65_536, seed=2, first_rg=0, codec="NONE"):
    """cfg2 (configs[1]) row groups [first_rg, first_rg + rows / rg_rows) of one logical file whose
    row group g is drawn from default_rng([seed, g]) (column a) and default_rng([seed + 1, g])
    (column b), so rank shards are a row-group partition of one file. Null masks are nudged so
    that no DELTA page has a non-null count = 1 (mod 256) or <= 1 (App. A Q1)."""
    import pyarrow as pa
    nrg = max(1, -(-rows // rg_rows))
    parts = []
    for g in range(first_rg, first_rg + nrg):
        n = min(rg_rows, rows - (g - first_rg) * rg_rows)
        rng = np.random.default_rng([seed, g])
        rng3 = np.random.default_rng([seed + 1, g])
        parts.append((np.cumsum(rng.integers(0, 2**16, n)) + g * 2**15 * rg_rows, rng.random(n) < 0.1,
                      rng3.random(n), rng3.random(n) < 0.1))
    a = np.concatenate([p[0] for p in parts]).astype(np.int64)
    m = np.concatenate([p[1] for p in parts])
    b = np.concatenate([p[2] for p in parts])
    m2 = np.concatenate([p[3] for p in parts])
    pages = m[: rows // page_rows * page_rows].reshape(-1, page_rows)
    nn = page_rows - pages.sum(1)
    for p in np.flatnonzero((nn % 256 == 1) | (nn <= 1)):
        k = np.flatnonzero(pages[p])[0]
        pages[p, k] = False  # one more non-null value
    t = pa.table({"a": pa.array(a, mask=m), "b": pa.array(b, mask=m2)})
    # SNAPPY pages are V1 (cfg5's page version): pyarrow stores an incompressible V2 values
    # section uncompressed with is_compressed=false, which the reference ignores (page_v2.go:125)
    return _write(t, use_dictionary=False, data_page_version="2.0" if codec == "NONE" else "1.0",
                  compression=codec, column_encoding={"a": "DELTA_BINARY_PACKED", "b": "PLAIN"},
                  max_rows_per_page=page_rows, row_group_size=rg_rows), (a, m, b, m2)


def cfg3_vocab(k=65_536, seed=4):
    """k distinct lowercase strings of length 4-28 (mean 16), as an Arrow string array."""
    import pyarrow as pa
    import pyarrow.compute as pc
    rng = np.random.default_rng(seed)
    lens = rng.integers(4, 29, 2 * k)
    chars = rng.integers(97, 123, int(lens.sum()), dtype=np.uint8)
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)
    cand = pa.Array.from_buffers(pa.string(), 2 * k, [None, pa.py_buffer(offs.tobytes()), pa.py_buffer(chars.tobytes())])
    u = pc.unique(cand)[:k]
    assert len(u) == k
    return u, rng


def gen_cfg3(rows=33_554_432, rg_rows=RG_ROWS, page_rows=65_536, seed=4, first_rg=0):
    """cfg3 (configs[2]): each row group uses all 65,536 entries (its first 65,536 rows are a
    permutation), so every dictionary has exactly 65,536 entries and pyarrow's index width is
    bit_width(65,535) = 16. Row group g draws from default_rng([seed, g])."""
    import pyarrow as pa
    vocab, _ = cfg3_vocab(seed=seed)
    k = len(vocab)
    nrg = max(1, -(-rows // rg_rows))
    idx = []
    for g in range(first_rg, first_rg + nrg):
        n = min(rg_rows, rows - (g - first_rg) * rg_rows)
        rng = np.random.default_rng([seed, g])
        idx.append(np.concatenate([rng.permutation(k), rng.integers(0, k, max(n - k, 0))])[:n])
    idx = np.concatenate(idx).astype(np.int32)
    t = pa.table({"s": vocab.take(pa.array(idx))}, schema=pa.schema([pa.field("s", pa.string(), nullable=False)]))
    return _write(t, use_dictionary=True, data_page_version="1.0", compression="NONE",
                  dictionary_pagesize_limit=8 << 20, max_rows_per_page=page_rows, row_group_size=rg_rows), (vocab, idx)


def gen_cfg4(records=16_777_216, rg_rows=RG_ROWS, page_rows=65_536, seed=5, first_rg=0):
    """cfg4 (configs[3]): l LIST<INT32> (5 % null lists, 5 % empty, else 1-8 elements, 5 % null
    elements) and m MAP<BYTE_ARRAY, INT64> (5 % null maps, 0-4 entries, keys from a 1,024-word
    vocabulary, dictionary-encoded; values 5 % null, PLAIN). Leaves: l.list.element (maxR 1,
    maxD 3), m.key_value.key (maxR 1, maxD 2), m.key_value.value (maxR 1, maxD 3)."""
    import pyarrow as pa
    import pyarrow.compute as pc
    rng = np.random.default_rng([seed, first_rg])
    n = records
    u = rng.random(n)
    lnull, lempty = u < 0.05, (u >= 0.05) & (u < 0.10)
    ln = rng.integers(1, 9, n)
    ln[lnull | lempty] = 0
    offs = np.concatenate([[0], np.cumsum(ln)]).astype(np.int32)
    ne = int(offs[-1])
    el = pa.array(rng.integers(-2**31, 2**31 - 1, ne, dtype=np.int64).astype(np.int32), mask=rng.random(ne) < 0.05)
    lcol = pa.ListArray.from_arrays(pa.array(offs), el, mask=pa.array(lnull))
    mnull = rng.random(n) < 0.05
    mn = rng.integers(0, 5, n)
    mn[mnull] = 0
    moffs = np.concatenate([[0], np.cumsum(mn)]).astype(np.int32)
    nm = int(moffs[-1])
    vocab = pc.unique(pa.array(["k%04d_" % i + "x" * int(i % 9) for i in range(1024)]))
    keys = vocab.take(pa.array(rng.integers(0, 1024, nm)))
    vals = pa.array(rng.integers(-2**62, 2**62, nm), mask=rng.random(nm) < 0.05)
    mcol = pa.MapArray.from_arrays(pa.array(moffs), keys, vals, mask=pa.array(mnull))
    return _write(pa.table({"l": lcol, "m": mcol}), data_page_version="1.0", compression="NONE",
                  use_dictionary=["m.key_value.key"], row_group_size=rg_rows, max_rows_per_page=page_rows), (lcol, mcol)


GENERATORS = {"cfg1": gen_cfg1, "cfg2": gen_cfg2, "cfg3": gen_cfg3, "cfg4": gen_cfg4}


CFG5_RG_ROWS = 3_906_250


def cfg5_template(rows=CFG5_RG_ROWS, seed=6, page_rows=65_536):
    """One cfg5 row group as a pyarrow file: 16 x INT32 RLE_DICTIONARY (256 distinct int32s,
    8-bit indices), 16 x INT64 DELTA_BINARY_PACKED (running sums of uniform [0, 2^16) steps),
    16 x DOUBLE PLAIN (uniform [0, 1)), 16 x INT64 PLAIN (uniform), REQUIRED, SNAPPY, V1, pages
    of 65,536 rows (DELTA page non-null counts then avoid 1 mod 256, App. A Q1)."""
    import pyarrow as pa
    rng = np.random.default_rng(seed)
    arrays, fields = [], []
    for j in range(16):
        d = rng.integers(-2**31, 2**31, 256, dtype=np.int64).astype(np.int32)
        arrays.append(pa.array(d[rng.integers(0, 256, rows)]))
        fields.append(pa.field(f"i32dict_{j}", pa.int32(), nullable=False))
    for j in range(16):
        arrays.append(pa.array(np.cumsum(rng.integers(0, 2**16, rows)).astype(np.int64)))
        fields.append(pa.field(f"i64delta_{j}", pa.int64(), nullable=False))
    for j in range(16):
        arrays.append(pa.array(rng.random(rows)))
        fields.append(pa.field(f"f64_{j}", pa.float64(), nullable=False))
    for j in range(16):
        arrays.append(pa.array(rng.integers(-2**62, 2**62, rows, dtype=np.int64)))
        fields.append(pa.field(f"i64_{j}", pa.int64(), nullable=False))
    t = pa.Table.from_arrays(arrays, schema=pa.schema(fields))
    enc = {f"i64delta_{j}": "DELTA_BINARY_PACKED" for j in range(16)}
    enc.update({f"f64_{j}": "PLAIN" for j in range(16)})
    enc.update({f"i64_{j}": "PLAIN" for j in range(16)})
    return _write(t, use_dictionary=[f"i32dict_{j}" for j in range(16)], column_encoding=enc, compression="snappy",
                  data_page_version="1.0", row_group_size=rows, max_rows_per_page=page_rows,
                  dictionary_pagesize_limit=1 << 20)


def replicate_row_groups(templates, n, shared=False):
    """A file of `n` row groups whose row group g is the (only) row group of templates[g mod T],
    byte for byte, behind a footer written here (rawpq's Thrift writer) with every column chunk's
    offsets moved to its copy. Decoding needs nothing else of the template footers.
    shared=True: each template's bytes are written once and every row group built from it points at
    them (the whole 256-row-group cfg5 file in two templates' bytes; a reader sees ordinary column
    chunks at the offsets the footer gives)."""
    import pyarrow.parquet as pq
    import rawpq as R
    metas = [pq.ParquetFile(io.BytesIO(t)).metadata for t in templates]
    m0 = metas[0]
    sch = m0.schema
    schema = [[(4, R.BIN, "schema"), (5, R.I32, len(sch))]]
    for c in range(len(sch)):
        col = sch.column(c)
        schema.append(R.schema_leaf(col.name, col.physical_type, "REQUIRED"))
    codec = {"UNCOMPRESSED": 0, "SNAPPY": 1, "GZIP": 2}
    out = bytearray(b"PAR1")
    rgs, total_rows = [], 0
    placed = {}  # shared: template index -> shift of its one copy
    for g in range(n):
        t, md = templates[g % len(templates)], metas[g % len(templates)].row_group(0)
        cols = [md.column(c) for c in range(md.num_columns)]
        start = [c.dictionary_page_offset if c.has_dictionary_page else c.data_page_offset for c in cols]
        lo = min(start)
        hi = max(s + c.total_compressed_size for s, c in zip(start, cols))
        if shared and g % len(templates) in placed:
            shift = placed[g % len(templates)]
        else:
            shift = len(out) - lo
            out += t[lo:hi]
            placed[g % len(templates)] = shift
        ccs = []
        for s0, c in zip(start, cols):
            md_f = [(1, R.I32, R.TYPES[c.physical_type]), (2, R.LIST, (R.I32, [R.ENC[e] for e in c.encodings])),
                    (3, R.LIST, (R.BIN, c.path_in_schema.split("."))), (4, R.I32, codec[c.compression]),
                    (5, R.I64, c.num_values), (6, R.I64, c.total_uncompressed_size),
                    (7, R.I64, c.total_compressed_size), (9, R.I64, c.data_page_offset + shift)]
            if c.has_dictionary_page:
                md_f.append((11, R.I64, c.dictionary_page_offset + shift))
            ccs.append([(2, R.I64, s0 + shift), (3, R.STRUCT, md_f)])
        rgs.append([(1, R.LIST, (R.STRUCT, ccs)), (2, R.I64, md.total_byte_size), (3, R.I64, md.num_rows)])
        total_rows += md.num_rows
    fmd = R.tstruct([(1, R.I32, 1), (2, R.LIST, (R.STRUCT, schema)), (3, R.I64, total_rows),
                     (4, R.LIST, (R.STRUCT, rgs)), (6, R.BIN, "cfg5 row-group templates replicated")])
    out += fmd + len(fmd).to_bytes(4, "little") + b"PAR1"
    return bytes(out)


def gen_cfg5_file(num_row_groups=256, rg_rows=CFG5_RG_ROWS, seed=6, templates=2):
    """The whole configs[4] file: `num_row_groups` row groups (256 x 3,906,250 rows = 1e9 rows of 64
    columns) over `templates` shared row-group templates (replicate_row_groups shared=True)."""
    tpl = [cfg5_template(rg_rows, seed=[seed, k]) for k in range(min(templates, num_row_groups))]
    return replicate_row_groups(tpl, num_row_groups, shared=True)


def gen_cfg5(rows=8 * CFG5_RG_ROWS, rg_rows=CFG5_RG_ROWS, seed=6, first_rg=0, templates=2):
    """cfg5 (configs[4]) row groups [first_rg, first_rg + rows / rg_rows): row group g is template
    (g mod templates), each template drawn from default_rng([seed, t])."""
    nrg = max(1, -(-rows // rg_rows))
    tpl = [cfg5_template(rg_rows, seed=[seed, (first_rg + k) % templates]) for k in range(min(templates, nrg))]
    order = [tpl[(first_rg + g) % templates - first_rg % templates if len(tpl) == templates else g % len(tpl)]
             for g in range(nrg)]
    return replicate_rows(order), None


def replicate_rows(templates_in_order):
    """replicate_row_groups over an explicit per-row-group template list."""
    uniq, idx = [], []
    for t in templates_in_order:
        for k, u in enumerate(uniq):
            if u is t:
                idx.append(k)
                break
        else:
            uniq.append(t)
            idx.append(len(uniq) - 1)
    if idx == [k % len(uniq) for k in range(len(idx))]:
        return replicate_row_groups(uniq, len(idx))
    return replicate_row_groups(list(templates_in_order), len(idx))
