"""Debug helper: walk page headers of a column chunk and report hybrid run statistics.
Standalone Thrift compact reader (debugging aid only, not used by tests or product)."""
import sys, io, struct
import pyarrow.parquet as pq

def uvar(b, i):
    x = s = 0
    while True:
        c = b[i]; i += 1
        x |= (c & 0x7f) << s; s += 7
        if c < 0x80: return x, i

def zz(u): return (u >> 1) ^ -(u & 1)

def read_struct(b, i):
    out = {}; last = 0
    while True:
        h = b[i]; i += 1
        if h == 0: return out, i
        t = h & 15; d = h >> 4
        if d: fid = last + d
        else: u, i = uvar(b, i); fid = zz(u)
        last = fid
        if t in (1, 2): out[fid] = (t == 1)
        elif t in (4, 5, 6): u, i = uvar(b, i); out[fid] = zz(u)
        elif t == 3: out[fid] = b[i]; i += 1
        elif t == 8: l, i = uvar(b, i); out[fid] = b[i:i+l]; i += l
        elif t == 12: out[fid], i = read_struct(b, i)
        elif t == 9:
            sz = b[i] >> 4; et = b[i] & 15; i += 1
            if sz == 15: sz, i = uvar(b, i)
            lst = []
            for _ in range(sz):
                if et == 12: v, i = read_struct(b, i)
                elif et in (5, 6, 4): u, i = uvar(b, i); v = zz(u)
                elif et == 8: l, i = uvar(b, i); v = b[i:i+l]; i += l
                else: raise ValueError(et)
                lst.append(v)
            out[fid] = lst
        else: raise ValueError(t)

def hybrid_runs(b, bw):
    i = 0; runs = []
    while i < len(b):
        h, i = uvar(b, i)
        if h & 1: g = h >> 1; runs.append(('bp', g * 8)); i += g * bw
        else: runs.append(('rle', h >> 1)); i += (bw + 7) // 8
    return runs

def pages(buf, rg=0, col=0):
    md = pq.ParquetFile(io.BytesIO(buf)).metadata.row_group(rg).column(col)
    off = md.dictionary_page_offset if md.has_dictionary_page else md.data_page_offset
    end = off + md.total_compressed_size
    while off < end:
        ph, j = read_struct(buf, off)
        yield ph, j
        off = j + ph[3]

if __name__ == '__main__':
    buf = open(sys.argv[1], 'rb').read()
    for ph, j in pages(buf):
        print(ph.get(1), {k: v for k, v in ph.items() if k not in (5, 8, 7)}, ph.get(5) or ph.get(8) or ph.get(7))
