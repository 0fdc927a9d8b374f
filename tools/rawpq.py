"""Minimal Parquet writer for hand-built pages (test-fixture tool, not product code).

pyarrow only emits DELTA_BINARY_PACKED with blockSize 256 / 4 miniblocks, so the
decoder paths for other block shapes (more than 4 miniblocks, blocks > 1024
values, miniblocks whose value count is not a multiple of 8 or 32), 10-byte
minDelta varints and arbitrary widths in unneeded trailing miniblocks are
reached only through streams written here. The encoder follows the format
specification (parquet-format Encodings.md, DELTA_BINARY_PACKED); the file
framing is the Thrift compact protocol (parquet.thrift field ids).
"""
import struct

import numpy as np

# ---------------------------------------------------------------- thrift compact


def uvar(x):
    out = bytearray()
    while True:
        b = x & 0x7F
        x >>= 7
        if x:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def zz64(v):
    return ((v << 1) ^ (v >> 63)) & 0xFFFFFFFFFFFFFFFF


I32, I64, BIN, LIST, STRUCT, BOOL = 5, 6, 8, 9, 12, 1


def tstruct(fields):
    """fields: [(id, type, value)] in increasing id order; value of STRUCT is a field list,
    of LIST is (elem_type, [values])."""
    out = bytearray()
    last = 0
    for fid, t, v in fields:
        if v is None:
            continue
        ct = t
        if t == BOOL:
            ct = 1 if v else 2
        d = fid - last
        if 0 < d <= 15:
            out.append((d << 4) | ct)
        else:
            out.append(ct)
            out += uvar(zz64(fid))
        last = fid
        out += tvalue(t, v)
    out.append(0)
    return bytes(out)


def tvalue(t, v):
    if t in (I32, I64):
        return uvar(zz64(v))
    if t == BIN:
        v = v.encode() if isinstance(v, str) else v
        return uvar(len(v)) + v
    if t == STRUCT:
        return tstruct(v)
    if t == BOOL:
        return b""
    if t == LIST:
        et, vals = v
        hdr = bytes([(len(vals) << 4) | et]) if len(vals) < 15 else bytes([0xF0 | et]) + uvar(len(vals))
        return hdr + b"".join(tvalue(et, x) for x in vals)
    raise ValueError(t)


# ---------------------------------------------------------------- encoders


def bitpack(vals, w):
    """LSB-first bit packing of non-negative ints at width w (len(vals) * w must be a multiple of 8)."""
    acc = 0
    for i, v in enumerate(vals):
        acc |= (int(v) & ((1 << w) - 1)) << (i * w)
    return acc.to_bytes(len(vals) * w // 8, "little") if w else b""


def hybrid_bitpacked(levels, bw):
    """RLE/bit-packing hybrid with one bit-packed run (levels padded to a multiple of 8)."""
    n = len(levels)
    g = (n + 7) // 8
    padded = list(levels) + [0] * (g * 8 - n)
    return uvar((g << 1) | 1) + bitpack(padded, bw)


def delta_encode(vals, bs=128, mbc=4, bits=64, trailing_width=0, min_delta_override=None, ref_single=False):
    """DELTA_BINARY_PACKED stream of `vals` (python ints, wrapped to `bits`).

    ref_single: a single value gets one empty block (minDelta MaxInt32, all widths 0), as the
    reference writer flushes it (deltaBitPackEncoder.write deltabp_encoder.go:139-144); the
    reader's look-ahead needs that header (App. A Q1).

    trailing_width: width byte written for miniblocks of the last block that hold no
    delta (the spec lets writers put anything there). min_delta_override: force every
    block's minDelta (widths are then computed for the wrapped differences)."""
    mask = (1 << bits) - 1
    sign = 1 << (bits - 1)

    def s(v):
        v &= mask
        return v - (1 << bits) if v & sign else v

    mbvc = bs // mbc
    out = bytearray(uvar(bs) + uvar(mbc) + uvar(len(vals)))
    if not vals:
        return bytes(out + uvar(0))
    out += uvar(zz64(s(vals[0])))
    if ref_single and len(vals) == 1:
        return bytes(out + uvar(zz64((1 << 31) - 1)) + bytes(mbc))
    deltas = [s(vals[i] - vals[i - 1]) for i in range(1, len(vals))]
    for b0 in range(0, len(deltas), bs):
        blk = deltas[b0:b0 + bs]
        md = min(blk) if min_delta_override is None else min_delta_override
        adj = [(d - md) & mask for d in blk]
        out += uvar(zz64(md))
        widths, bodies = [], []
        for m in range(mbc):
            mb = adj[m * mbvc:(m + 1) * mbvc]
            if not mb:
                widths.append(trailing_width)
                continue
            w = max(int(x).bit_length() for x in mb)
            widths.append(w)
            mb = mb + [0] * (mbvc - len(mb))
            if (mbvc * w) % 8:
                pad = (8 - (mbvc * w) % 8)
                body = bitpack(mb + [0] * pad, w)  # round up to whole bytes
                body = body[: (mbvc * w + 7) // 8]
            else:
                body = bitpack(mb, w)
            bodies.append(body)
        out += bytes(widths)
        for body in bodies:
            out += body
    return bytes(out)


# ---------------------------------------------------------------- file framing

TYPES = {"INT32": 1, "INT64": 2, "DOUBLE": 5, "BYTE_ARRAY": 6}
ENC = {"PLAIN": 0, "RLE": 3, "DELTA_BINARY_PACKED": 5, "DELTA_LENGTH_BYTE_ARRAY": 6, "DELTA_BYTE_ARRAY": 7}


def page_v1(values_bytes, num_values, encoding, def_bytes=b""):
    """DATA_PAGE (V1): [def levels with u32 length prefix] + values."""
    body = (struct.pack("<I", len(def_bytes)) + def_bytes if def_bytes else b"") + values_bytes
    dph = [(1, I32, num_values), (2, I32, ENC[encoding]), (3, I32, ENC["RLE"]), (4, I32, ENC["RLE"])]
    hdr = tstruct([(1, I32, 0), (2, I32, len(body)), (3, I32, len(body)), (5, STRUCT, dph)])
    return hdr + body


def page_v2(values_bytes, num_values, num_nulls, num_rows, encoding, def_bytes=b""):
    body = def_bytes + values_bytes
    dph = [(1, I32, num_values), (2, I32, num_nulls), (3, I32, num_rows), (4, I32, ENC[encoding]),
           (5, I32, len(def_bytes)), (6, I32, 0), (7, BOOL, False)]
    hdr = tstruct([(1, I32, 3), (2, I32, len(body)), (3, I32, len(body)), (8, STRUCT, dph)])
    return hdr + body


def write_file(columns, row_groups, codec=0):
    """columns: [(name, type, optional)]; row_groups: [(num_rows, [[page bytes, ...] per column],
    [num_values per column])]; codec: 0 UNCOMPRESSED, 1 SNAPPY (pages already compressed).
    Returns the file bytes."""
    out = bytearray(b"PAR1")
    rgs = []
    for num_rows, col_pages, col_nv in row_groups:
        ccs = []
        total = 0
        for (name, typ, opt), pages, nv in zip(columns, col_pages, col_nv):
            off = len(out)
            for p in pages:
                out += p
            size = len(out) - off
            total += size
            md = [(1, I32, TYPES[typ]), (2, LIST, (I32, [0, 3, 5])), (3, LIST, (BIN, [name])), (4, I32, codec),
                  (5, I64, nv), (6, I64, size), (7, I64, size), (9, I64, off)]
            ccs.append([(2, I64, off), (3, STRUCT, md)])
        rgs.append([(1, LIST, (STRUCT, ccs)), (2, I64, total), (3, I64, num_rows)])
    schema = [[(4, BIN, "schema"), (5, I32, len(columns))]]
    for name, typ, opt in columns:
        schema.append([(1, I32, TYPES[typ]), (3, I32, 1 if opt else 0), (4, BIN, name)])
    fmd = tstruct([(1, I32, 1), (2, LIST, (STRUCT, schema)), (3, I64, sum(r[0] for r in row_groups)),
                   (4, LIST, (STRUCT, rgs)), (6, BIN, "rawpq fixture writer")])
    out += fmd + struct.pack("<I", len(fmd)) + b"PAR1"
    return bytes(out)


def delta_column_file(pages_vals, bs, mbc, typ="INT64", v2=False, rg_split=None, **kw):
    """A one-column REQUIRED file whose pages are DELTA streams of the given value lists."""
    bits = 64 if typ == "INT64" else 32
    pages = []
    for vals in pages_vals:
        st = delta_encode(vals, bs, mbc, bits, **kw)
        pages.append(page_v2(st, len(vals), 0, len(vals), "DELTA_BINARY_PACKED") if v2
                     else page_v1(st, len(vals), "DELTA_BINARY_PACKED"))
    groups = rg_split or [len(pages)]
    rgs, k = [], 0
    for g in groups:
        ps, vs = pages[k:k + g], pages_vals[k:k + g]
        n = sum(len(v) for v in vs)
        rgs.append((n, [ps], [n]))
        k += g
    return write_file([("a", typ, False)], rgs)


def random_walk(rng, n, step_bits, signed=True):
    lo = -(1 << (step_bits - 1)) if signed else 0
    d = rng.integers(lo, 1 << (step_bits - 1), n, dtype=np.int64)
    return [int(x) for x in np.cumsum(d)]


def dlba_stream(lens, payload, bs=128, mbc=4, **kw):
    """DELTA_LENGTH_BYTE_ARRAY values section: DELTA INT32 lengths, then the bytes."""
    return delta_encode(list(lens), bs, mbc, 32, **kw) + bytes(payload)


def dba_stream(prefixes, suffix_lens, payload, bs=128, mbc=4, **kw):
    """DELTA_BYTE_ARRAY values section: DELTA prefix lengths, DELTA suffix lengths, suffix bytes."""
    return delta_encode(list(prefixes), bs, mbc, 32, **kw) + delta_encode(list(suffix_lens), bs, mbc, 32, **kw) + bytes(payload)


def dba_encode(values):
    """(prefix lengths, suffix lengths, suffix bytes) of a list of bytes values."""
    pre, sl, pay, prev = [], [], bytearray(), b""
    for v in values:
        k = 0
        while k < min(len(v), len(prev)) and v[k] == prev[k]:
            k += 1
        pre.append(k)
        sl.append(len(v) - k)
        pay += v[k:]
        prev = v
    return pre, sl, bytes(pay)


def ba_column_file(pages, encoding, v2=False):
    """A one-column REQUIRED BYTE_ARRAY file: pages = [(values section bytes, num_values)]."""
    ps = [page_v2(st, n, 0, n, encoding) if v2 else page_v1(st, n, encoding) for st, n in pages]
    n = sum(k for _, k in pages)
    return write_file([("s", "BYTE_ARRAY", False)], [(n, [ps], [n])])


# ---------------------------------------------------------------- raw snappy blocks
# Element encoders follow the snappy block format (format_description.txt: tag & 3 = literal /
# copy with 1-, 2- or 4-byte offset; literal lengths above 60 in 1-4 extra bytes), so streams
# with chosen element kinds, far offsets and deliberate corruption can be built.


def sn_literal(data, extra=None):
    """A literal element; `extra` forces 1-4 length bytes (else the shortest form)."""
    n = len(data) - 1
    if extra is None:
        extra = 0 if n < 60 else 1 if n < 1 << 8 else 2 if n < 1 << 16 else 3 if n < 1 << 24 else 4
    if extra == 0:
        return bytes([n << 2]) + bytes(data)
    return bytes([(59 + extra) << 2]) + n.to_bytes(extra, "little") + bytes(data)


def sn_copy(off, length, kind):
    """A copy element: kind 1 (length 4-11, offset < 2048), 2 (offset < 65536) or 4."""
    if kind == 1:
        assert 4 <= length <= 11 and off < 2048
        return bytes([1 | ((length - 4) << 2) | ((off >> 8) << 5), off & 0xFF])
    assert 1 <= length <= 64
    if kind == 2:
        return bytes([2 | ((length - 1) << 2)]) + off.to_bytes(2, "little")
    return bytes([3 | ((length - 1) << 2)]) + off.to_bytes(4, "little")


def snappy_block(dlen, elements):
    return uvar(dlen) + b"".join(elements)


def snappy_compress(data, rng=None, min_match=4, max_lit=None):
    """Greedy LZ77 into snappy elements with no window limit (offsets up to the whole input,
    copy-4 past 64 KiB). With `rng` the copy kind, copy length split and literal length
    form vary at random so every element encoding occurs."""
    data = bytes(data)
    n = len(data)
    last = {}
    out, lit = [], bytearray()

    def flush_lit():
        k = 0
        while k < len(lit):
            m = len(lit) - k if max_lit is None else min(max_lit, len(lit) - k)
            extra = None
            if rng is not None and m - 1 >= 60 and rng.random() < 0.3:
                extra = int(rng.integers(1, 5))
                if m - 1 >= 1 << (8 * extra):
                    extra = None
            out.append(sn_literal(lit[k:k + m], extra))
            k += m
        lit.clear()

    i = 0
    while i < n:
        key = data[i:i + min_match]
        j = last.get(key) if len(key) == min_match else None
        if len(key) == min_match:
            last[key] = i
        if j is None:
            lit.append(data[i])
            i += 1
            continue
        off = i - j
        L = min_match
        while i + L < n and data[i + L] == data[j + L]:
            L += 1
        flush_lit()
        k = 0
        while k < L:
            cap = 64 if rng is None else int(rng.integers(4, 65))
            m = min(cap, L - k)  # a tail shorter than 4 is still a valid copy (kinds 2 and 4)
            kinds = [4]
            if off < 65536:
                kinds.append(2)
            if 4 <= m <= 11 and off < 2048:
                kinds.append(1)
            kind = kinds[-1] if rng is None else kinds[int(rng.integers(0, len(kinds)))]
            out.append(sn_copy(off, m, kind))
            k += m
        for t in range(i + 1, min(i + L, n - min_match + 1)):
            last[data[t:t + min_match]] = t
        i += L
    flush_lit()
    return snappy_block(n, out)


def page_v1c(values_bytes, num_values, encoding, def_bytes=b"", compress=None):
    """DATA_PAGE (V1) whose whole body goes through `compress` (bytes -> bytes)."""
    body = (struct.pack("<I", len(def_bytes)) + def_bytes if def_bytes else b"") + values_bytes
    cbody = compress(body) if compress else body
    dph = [(1, I32, num_values), (2, I32, ENC[encoding]), (3, I32, ENC["RLE"]), (4, I32, ENC["RLE"])]
    hdr = tstruct([(1, I32, 0), (2, I32, len(body)), (3, I32, len(cbody)), (5, STRUCT, dph)])
    return hdr + cbody


def page_v2c(values_bytes, num_values, num_nulls, num_rows, encoding, def_bytes=b"", compress=None):
    """DATA_PAGE_V2: level bytes raw, values through `compress` (page_v2.go:112-127)."""
    cvals = compress(values_bytes) if compress else values_bytes
    dph = [(1, I32, num_values), (2, I32, num_nulls), (3, I32, num_rows), (4, I32, ENC[encoding]),
           (5, I32, len(def_bytes)), (6, I32, 0), (7, BOOL, True)]
    hdr = tstruct([(1, I32, 3), (2, I32, len(def_bytes) + len(values_bytes)),
                   (3, I32, len(def_bytes) + len(cvals)), (8, STRUCT, dph)])
    return hdr + def_bytes + cvals


# ---------------------------------------------------------------- reference-writer-style files
# The reference writer (fraugster/parquet-go) emits every hybrid stream as ONE bit-packed run
# (hybridEncoder.bpEncode hybrid_encoder.go:55-70), level bit width bits.Len16(max)
# (helpers.go:262-290), dictionary index width bits.Len(len(dict)) (page_v1.go:185,
# page_v2.go:200) and DELTA blocks of 128 values in 4 miniblocks. The helpers below build pages
# in that shape (and nested schemas, dictionary pages, page CRCs) so the GPU's dictionary and
# level paths see the reference's own stream layout.

TYPES.update({"BOOLEAN": 0, "INT96": 3, "FLOAT": 4, "FIXED_LEN_BYTE_ARRAY": 7})
ENC.update({"PLAIN_DICTIONARY": 2, "RLE_DICTIONARY": 8})
REP = {"REQUIRED": 0, "OPTIONAL": 1, "REPEATED": 2}


def hybrid_ref(vals, bw):
    """hybridEncoder: one bit-packed run of all values (nothing at bit width 0)."""
    return b"" if bw == 0 else hybrid_bitpacked(list(vals), bw)


def levels_v1_ref(levels, max_level):
    """encodeLevelsV1: u32 byte length + hybrid_ref at bits.Len16(max)."""
    st = hybrid_ref(levels, int(max_level).bit_length())
    return struct.pack("<I", len(st)) + st


def plain_encode(typ, vals, type_length=0):
    """PLAIN values section (type_*.go encoders): LE fixed width, BOOLEAN LSB-first bits,
    BYTE_ARRAY u32 length + bytes, FIXED_LEN_BYTE_ARRAY raw bytes."""
    if typ == "INT32":
        return np.asarray(vals, "<i4").tobytes()
    if typ == "INT64":
        return np.asarray(vals, "<i8").tobytes()
    if typ == "FLOAT":
        return np.asarray(vals, "<f4").tobytes()
    if typ == "DOUBLE":
        return np.asarray(vals, "<f8").tobytes()
    if typ == "BOOLEAN":
        bits = np.zeros(-(-len(vals) // 8) * 8, np.uint8)
        bits[:len(vals)] = np.asarray(vals, bool)
        return np.packbits(bits, bitorder="little").tobytes()
    if typ == "BYTE_ARRAY":
        return b"".join(struct.pack("<I", len(v)) + bytes(v) for v in vals)
    if typ == "FIXED_LEN_BYTE_ARRAY":
        assert all(len(v) == type_length for v in vals)
        return b"".join(bytes(v) for v in vals)
    raise ValueError(typ)


def _page(ptype, body, hdr_field, hdr_struct, crc=False, usize=None):
    import zlib
    f = [(1, I32, ptype), (2, I32, len(body) if usize is None else usize), (3, I32, len(body))]
    if crc:
        c = zlib.crc32(body) & 0xFFFFFFFF
        f.append((4, I32, c - (1 << 32) if c >= 1 << 31 else c))
    f.append((hdr_field, STRUCT, hdr_struct))
    return tstruct(f) + body


def dict_page_ref(typ, entries, type_length=0, crc=False):
    """DICTIONARY_PAGE with PLAIN entries (page_dict.go:74-136)."""
    return _page(2, plain_encode(typ, entries, type_length), 7, [(1, I32, len(entries)), (2, I32, ENC["PLAIN"])], crc)


def data_page_v1_ref(num_values, encoding, values_section, def_levels=None, max_def=0, rep_levels=None, max_rep=0,
                     crc=False):
    """DATA_PAGE: [rep: u32 + hybrid] [def: u32 + hybrid] values (page_v1.go:124-231)."""
    body = b""
    if max_rep > 0:
        body += levels_v1_ref(rep_levels, max_rep)
    if max_def > 0:
        body += levels_v1_ref(def_levels, max_def)
    body += values_section
    dph = [(1, I32, num_values), (2, I32, ENC[encoding]), (3, I32, ENC["RLE"]), (4, I32, ENC["RLE"])]
    return _page(0, body, 5, dph, crc)


def data_page_v2_ref(num_values, num_nulls, num_rows, encoding, values_section, def_levels=None, max_def=0,
                     rep_levels=None, max_rep=0, crc=False):
    """DATA_PAGE_V2: rep and def hybrid streams without length prefix, then values (page_v2.go:133-255)."""
    rep = hybrid_ref(rep_levels, int(max_rep).bit_length()) if max_rep > 0 else b""
    dfn = hybrid_ref(def_levels, int(max_def).bit_length()) if max_def > 0 else b""
    body = rep + dfn + values_section
    dph = [(1, I32, num_values), (2, I32, num_nulls), (3, I32, num_rows), (4, I32, ENC[encoding]),
           (5, I32, len(dfn)), (6, I32, len(rep)), (7, BOOL, False)]
    return _page(3, body, 8, dph, crc)


def dict_values_section(indices, dict_len):
    """RLE_DICTIONARY values section as the reference writes it: 1 byte bit width
    bits.Len(len(dict)), then one bit-packed run (dictEncoder, type_dict.go)."""
    bw = int(dict_len).bit_length()
    return bytes([bw]) + hybrid_ref(indices, bw)


def schema_group(name, rep, num_children):
    return [(3, I32, REP[rep]), (4, BIN, name), (5, I32, num_children)]


def schema_leaf(name, typ, rep, type_length=None):
    return [(1, I32, TYPES[typ]), (2, I32, type_length), (3, I32, REP[rep]), (4, BIN, name)]


def write_file_schema(schema, leaves, row_groups, codec=0):
    """schema: SchemaElement field lists in depth-first order (root first, with num_children);
    leaves: [(dotted path, type)] in column order; row_groups: [(num_rows, [(pages, num_values,
    has_dict) per leaf])] where pages are whole page byte strings (a dictionary page first when
    has_dict). Returns the file bytes."""
    out = bytearray(b"PAR1")
    rgs = []
    for num_rows, chunks in row_groups:
        ccs, total = [], 0
        for (path, typ), (pages, nv, has_dict) in zip(leaves, chunks):
            off = len(out)
            data_off = off
            for k, p in enumerate(pages):
                if k == 1 and has_dict:
                    data_off = len(out)
                out += p
            size = len(out) - off
            total += size
            md = [(1, I32, TYPES[typ]), (2, LIST, (I32, [0, 3, 8] if has_dict else [0, 3])),
                  (3, LIST, (BIN, path.split("."))), (4, I32, codec), (5, I64, nv), (6, I64, size), (7, I64, size),
                  (9, I64, data_off)]
            if has_dict:
                md.append((11, I64, off))
            ccs.append([(2, I64, off), (3, STRUCT, md)])
        rgs.append([(1, LIST, (STRUCT, ccs)), (2, I64, total), (3, I64, num_rows)])
    fmd = tstruct([(1, I32, 1), (2, LIST, (STRUCT, schema)), (3, I64, sum(r[0] for r in row_groups)),
                   (4, LIST, (STRUCT, rgs)), (6, BIN, "rawpq reference-style writer")])
    out += fmd + struct.pack("<I", len(fmd)) + b"PAR1"
    return bytes(out)


def crc_probe_chunk(pages):
    """A bare chunk of DATA_PAGE (V1) pages with given bodies and stored checksums [(body, crc)], for
    the device CRC32 check: (bytes, [pqgpu.ChunkMeta]) with the chunk at offset 0."""
    import pqgpu
    out = bytearray()
    for body, c in pages:
        c &= 0xFFFFFFFF
        dph = [(1, I32, 0), (2, I32, ENC["PLAIN"]), (3, I32, ENC["RLE"]), (4, I32, ENC["RLE"])]
        out += tstruct([(1, I32, 0), (2, I32, len(body)), (3, I32, len(body)),
                        (4, I32, c - (1 << 32) if c >= 1 << 31 else c), (5, STRUCT, dph)]) + body
    m = pqgpu.ChunkMeta(TYPES["INT32"], 0, 0, len(out), 0, -1, 0, 0)
    return bytes(out), [m]
