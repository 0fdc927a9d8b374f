// pagewalk.hip — the on-device page index: readPages' page-header loop
// (chunk_reader.go:182-263) with the Thrift compact decode of every PageHeader (readThrift,
// helpers.go:103-109; parquet/parquet.go PageHeader.Read) over column-chunk bytes resident in HBM,
// the CRC32 check of readPageBlock (chunk_reader.go:173-177: crc32.ChecksumIEEE of the page block
// against PageHeader.Crc), and the device-to-device gather of UNCOMPRESSED page bodies into a
// batch's page region.
//
//   k_page_walk    one wavefront per column chunk. The header chain is serial (page k+1 starts
//                  after page k's header and block), so the whole wave walks it in lock step:
//                  the bytes around the cursor sit in a 256-byte register window (lane l holds
//                  4 bytes) and every byte of the Thrift decode is one readlane at a wave-uniform
//                  index. Page k's fields land in lane k mod 64's registers; every 64 pages the
//                  wave reserves 64 consecutive table entries with one atomic and stores them
//                  coalesced, so a chunk's entries are in page order within the table.
//                  Only the valid case is walked: anything the walk cannot take (a Thrift error,
//                  a negative block size, a block past the resident bytes, nesting deeper than
//                  kIxDepth, a full table) marks the chunk IX_FALLBACK and the host walks it
//                  itself, so errors keep the host's class, message and position.
//   k_page_crc     one 256-thread workgroup per page with a checksum (grid-stride over the table):
//                  thread t takes a contiguous quarter-KiB-scale segment of the block and runs
//                  slicing-by-4 CRC32 (IEEE, reflected 0xEDB88320) from four LDS tables; the
//                  segment checksums combine by crc(A||B) = (x^(8|B|) mod P)·crc(A) xor crc(B)
//                  (zlib's crc32_combine: the multiply is a 32-step carry-less product modulo P,
//                  x^(8n) from the squares x^(2^k)), XOR-reduced over the workgroup.
//   k_page_gather  one workgroup per UNCOMPRESSED page: the block is copied into the batch's page
//                  region (16-B aligned destination, funnel-shifted 16-B stores) with 64 zero
//                  bytes after it, the layout every decode kernel reads.
#include <hip/hip_runtime.h>
#include <string.h>

#include <algorithm>

#include "dev_util.h"
#include "kernels.h"

namespace pq {

constexpr uint32_t kIxDepth = 24;  // Thrift nesting the walk follows (the host allows 64: deeper -> host)
constexpr uint32_t kCrcPoly = 0xedb88320u;
static_assert(kIxArgChunks * sizeof(PageIxChunk) + 64 <= 4096, "chunk table must fit the kernel arguments");

// ---------------------------------------------------------------------------
// Thrift compact decode from a wave-wide register window
// ---------------------------------------------------------------------------
enum { TC_STOP = 0, TC_TRUE = 1, TC_FALSE = 2, TC_BYTE = 3, TC_I16 = 4, TC_I32 = 5, TC_I64 = 6, TC_DOUBLE = 7,
       TC_BINARY = 8, TC_LIST = 9, TC_SET = 10, TC_MAP = 11, TC_STRUCT = 12 };

// Cursor over the bytes [0, len) of `buf` (one chunk's span of the resident bytes, so positions
// are 32-bit: the cursor checks compile to scalar compares); lane l's `w` holds bytes
// [base + 4l, +4). Every member is wave-uniform.
struct TWin {
  const uint8_t *buf;
  uint32_t len;
  uint32_t base;
  uint32_t w;
  uint32_t i;   // next byte (span-relative)
  bool err;
};

DEV void twin_load(TWin &t, uint32_t at) {
  t.base = at & ~3u;
  const uint64_t p = (uint64_t)t.base + 4 * lane_id();
  uint32_t w = 0;
  if (p + 4 <= t.len) {
    w = *(const uint32_t *)(t.buf + p);
  } else {
    for (int k = 0; k < 4; k++)
      if (p + k < t.len) w |= (uint32_t)t.buf[p + k] << (8 * k);
  }
  t.w = w;
}

DEV bool tbyte(TWin &t, uint32_t &b) {
  if (t.err || t.i >= t.len) { t.err = true; return false; }
  if (t.i - t.base >= 256u) twin_load(t, t.i);  // unsigned: also when i < base
  const uint32_t r = t.i - t.base;
  b = (rdlane(t.w, r >> 2) >> (8 * (r & 3))) & 0xffu;
  t.i++;
  return true;
}

// ThriftReader::uvarint (format.cpp): bits past 64 are dropped, the varint may be any length
DEV uint64_t tuvarint(TWin &t) {
  uint64_t x = 0;
  uint32_t s = 0;
  for (;;) {
    uint32_t b;
    if (!tbyte(t, b)) return 0;
    if (s < 64) x |= (uint64_t)(b & 0x7f) << s;
    if (!(b & 0x80)) return x;
    s += 7;
  }
}
DEV int32_t ti32(TWin &t) {
  const uint32_t u = (uint32_t)tuvarint(t);
  return (int32_t)(u >> 1) ^ -(int32_t)(u & 1);
}

// ThriftReader::field: false at STOP or on an error
DEV bool tfield(TWin &t, int32_t &last, int32_t &id, int32_t &type) {
  uint32_t b;
  if (!tbyte(t, b)) return false;
  if ((b & 0x0f) == TC_STOP) return false;
  const int32_t mod = (int32_t)(b >> 4);
  id = mod ? (int32_t)(int16_t)(last + mod) : (int32_t)(int16_t)ti32(t);
  if (t.err) return false;
  last = id;
  type = (int32_t)(b & 0x0f);
  if (type > TC_STRUCT) { t.err = true; return false; }
  return true;
}

// ThriftReader::skip(type, depth) without recursion: containers are frames of an LDS stack
// (wave-uniform, written identically by every lane).
struct TFrame {
  int64_t rem;     // list/set: elements left; map: keys + values left; struct: unused
  int32_t last;    // struct: last field id
  uint8_t kind;    // TC_LIST / TC_MAP / TC_STRUCT
  uint8_t et;      // list element type; map: key type << 4 | value type
  uint8_t depth;   // the container's own depth
  uint8_t pad;
};

DEV void tskip(TWin &t, int32_t ty, uint32_t depth, TFrame *stk) {
  uint32_t sp = 0;
  bool have = true;
  while (!t.err) {
    if (have) {
      have = false;
      if (depth > 64) { t.err = true; break; }
      uint32_t b;
      switch (ty) {
        case TC_TRUE: case TC_FALSE: case TC_BYTE: tbyte(t, b); break;
        case TC_I16: case TC_I32: case TC_I64: tuvarint(t); break;
        case TC_DOUBLE:
          if (t.len - t.i < 8) t.err = true; else t.i += 8;
          break;
        case TC_BINARY: {
          const int32_t n = (int32_t)tuvarint(t);
          if (t.err) break;
          if (n < 0 || (uint32_t)n > t.len - t.i) { t.err = true; break; }
          t.i += n;
          break;
        }
        case TC_LIST: case TC_SET: {
          if (!tbyte(t, b)) break;
          int32_t sz = (int32_t)((b >> 4) & 0x0f);
          if (sz == 15) sz = (int32_t)tuvarint(t);
          if (t.err || sz < 0 || (b & 0x0f) > TC_STRUCT) { t.err = true; break; }
          if (sp >= kIxDepth) { t.err = true; break; }  // deeper than the walk follows: host
          stk[sp] = TFrame{sz, 0, TC_LIST, (uint8_t)(b & 0x0f), (uint8_t)depth, 0};
          sp++;
          break;
        }
        case TC_MAP: {
          const int32_t n = (int32_t)tuvarint(t);
          if (t.err) break;
          if (n < 0) { t.err = true; break; }
          if (n == 0) break;
          if (!tbyte(t, b)) break;
          if (sp >= kIxDepth) { t.err = true; break; }
          stk[sp] = TFrame{2 * (int64_t)n, 0, TC_MAP, (uint8_t)b, (uint8_t)depth, 0};
          sp++;
          break;
        }
        case TC_STRUCT:
          if (sp >= kIxDepth) { t.err = true; break; }
          stk[sp] = TFrame{0, 0, TC_STRUCT, 0, (uint8_t)depth, 0};
          sp++;
          break;
        default: t.err = true;
      }
      wave_lds_sync();
    }
    if (t.err || sp == 0) break;
    TFrame f = stk[sp - 1];
    if (f.kind == TC_STRUCT) {
      int32_t id, fty;
      const bool more = tfield(t, f.last, id, fty);
      stk[sp - 1].last = f.last;
      wave_lds_sync();
      if (!more) { if (!t.err) sp--; continue; }
      if (fty != TC_TRUE && fty != TC_FALSE) { ty = fty; depth = f.depth + 1u; have = true; }
      continue;
    }
    if (f.rem == 0) { sp--; continue; }
    f.rem--;
    stk[sp - 1].rem = f.rem;
    wave_lds_sync();
    // map: keys and values alternate; with 2n entries left before the decrement a key comes first
    ty = f.kind == TC_LIST ? (int32_t)f.et : ((f.rem & 1) ? (int32_t)(f.et >> 4) : (int32_t)(f.et & 0x0f));
    depth = f.depth + 1u;
    have = true;
  }
}

DEV void tskip_field(TWin &t, int32_t ty, TFrame *stk) {
  if (ty != TC_TRUE && ty != TC_FALSE) tskip(t, ty, 1, stk);
}

// arr[k] = v with constant indices only, so the header stays in registers (a dynamically indexed
// member array would put the whole entry in scratch memory)
template <int N>
DEV void set_field(int32_t (&arr)[N], int32_t k, int32_t v) {
#pragma unroll
  for (int j = 0; j < N; j++)
    if (k == j) arr[j] = v;
}

// ParsePageHeader (format.cpp; the generated PageHeader.Read with its required-field checks)
DEV bool parse_page_header(TWin &t, PageIxEntry &h, TFrame *stk) {
  int32_t last = 0, id, ty;
  bool st = false, su = false, sc = false;
  h.type = h.usize = h.csize = h.crc = 0;
  h.flags = IXF_COMPRESSED;  // DataPageHeaderV2.is_compressed defaults to true
  for (int k = 0; k < 4; k++) h.dph[k] = 0;
  h.dict[0] = h.dict[1] = 0;
  for (int k = 0; k < 6; k++) h.dph2[k] = 0;
  while (tfield(t, last, id, ty)) {
    if (id == 1 && ty == TC_I32) { h.type = ti32(t); st = true; }
    else if (id == 2 && ty == TC_I32) { h.usize = ti32(t); su = true; }
    else if (id == 3 && ty == TC_I32) { h.csize = ti32(t); sc = true; }
    else if (id == 4 && ty == TC_I32) { h.crc = ti32(t); h.flags |= IXF_CRC; }
    else if (id == 5 && ty == TC_STRUCT) {
      h.flags |= IXF_DPH;
      int32_t l2 = 0, i2, t2;
      uint32_t set = 0;
      while (tfield(t, l2, i2, t2)) {
        if (i2 >= 1 && i2 <= 4 && t2 == TC_I32) { set_field(h.dph, i2 - 1, ti32(t)); set |= 1u << i2; }
        else tskip_field(t, t2, stk);
      }
      if (!t.err && set != 0x1e) t.err = true;
    } else if (id == 7 && ty == TC_STRUCT) {
      h.flags |= IXF_DICT;
      int32_t l2 = 0, i2, t2;
      uint32_t set = 0;
      while (tfield(t, l2, i2, t2)) {
        if (i2 >= 1 && i2 <= 2 && t2 == TC_I32) { set_field(h.dict, i2 - 1, ti32(t)); set |= 1u << i2; }
        else tskip_field(t, t2, stk);
      }
      if (!t.err && set != 0x6) t.err = true;
    } else if (id == 8 && ty == TC_STRUCT) {
      h.flags |= IXF_DPH2;
      int32_t l2 = 0, i2, t2;
      uint32_t set = 0;
      while (tfield(t, l2, i2, t2)) {
        if (t2 == TC_I32 && i2 >= 1 && i2 <= 6) {
          const int32_t v = ti32(t);
          set |= 1u << i2;
          // PageHeader field order 1..6: num_values, num_nulls, num_rows, encoding, def_len, rep_len
          set_field(h.dph2, i2 - 1, v);
        } else if (i2 == 7 && (t2 == TC_TRUE || t2 == TC_FALSE)) {
          h.flags = t2 == TC_TRUE ? (h.flags | IXF_COMPRESSED) : (h.flags & ~IXF_COMPRESSED);
        } else tskip_field(t, t2, stk);
      }
      if (!t.err && set != 0x7e) t.err = true;
    } else tskip_field(t, ty, stk);
  }
  if (!t.err && !(st && su && sc)) t.err = true;
  return !t.err;
}

// One wavefront per chunk: the header chain of readPages.
// The chunk table travels in the kernel arguments (kIxArgChunks per launch); results go to `res`.
struct IxChunkArgs {
  PageIxChunk c[kIxArgChunks];
};

__global__ void __launch_bounds__(64) k_page_walk(const uint8_t *buf_in, int64_t len, int64_t file_off,
                                                  const IxChunkArgs args, uint32_t chunk0, uint4 *res_in,
                                                  PageIxEntry *table_in, uint32_t *table_n, uint32_t table_cap,
                                                  uint32_t gen, uint32_t test_skip) {
  __shared__ TFrame stk[kIxDepth];
  const uint8_t *buf = gp(buf_in);
  PageIxEntry *table = gp(table_in);
  const uint32_t c = chunk0 + blockIdx.x, lane = lane_id();
  const PageIxChunk ch = args.c[blockIdx.x];
  // the chunk's span of the resident bytes: from its first header (or its data pages, when they
  // come first) to the end, at most 4 GiB - 1 (a walk that needs more falls back)
  const int64_t first = (ch.data_off >= 0 ? min(ch.start, ch.data_off) : ch.start) - file_off;
  const int64_t cb = first < 0 ? 0 : min(first, len);
  TWin t;
  t.buf = buf + cb;
  t.len = (uint32_t)min(len - cb, (int64_t)0xffffffffll);
  t.base = 0xfffff000u;  // no window yet
  t.w = 0;
  t.err = false;
  int64_t off = ch.start, count = 0;
  uint32_t seq = 0, flushed = 0, status = IX_OK;
  bool had_dict = false;
  PageIxEntry mine;  // page seq of this lane within the current group of 64
  auto flush = [&](uint32_t n) -> bool {
    uint32_t at = 0;
    if (lane == 0) at = atomicAdd(table_n, n);
    at = sgpr(__shfl(at, 0));
    if ((uint64_t)at + n > table_cap) return false;
    // test_skip (PQ_IX_TEST_SKIP_STORE, diagnostic build): chunk test_skip reserves its slots but stores
    // nothing, as if its stores were lost; the host must not trust what the slots hold
    if (lane < n && c != test_skip) table[at + lane] = mine;
    return true;
  };
  while (ch.total - count > 0) {
    const int64_t rel = off - file_off - cb;
    if (rel < 0 || rel >= (int64_t)t.len) { status = IX_FALLBACK; break; }
    PageIxEntry h;
    t.i = (uint32_t)rel;
    t.err = false;
    if (!parse_page_header(t, h, stk)) { status = IX_FALLBACK; break; }
    const int64_t hl = (int64_t)(t.i - (uint32_t)rel);
    off += hl;
    count += hl;
    // readPageBlock: the whole block must be resident (a short block is the host's error)
    if (h.csize < 0 || h.usize < 0 || off - file_off + (int64_t)h.csize > len) { status = IX_FALLBACK; break; }
    h.hdr_off = off - hl;
    h.hdr_len = (int32_t)hl;
    h.chunk = c;
    h.seq = seq;
    h.gen = gen;
    h.pad = 0;
    if (lane == (seq & 63)) mine = h;
    off += h.csize;
    count += h.csize;
    // a second dictionary page is the host's error ("there should be only one dictionary"); it also
    // bounds the walk: only a dictionary page seeks, so without one `count` grows every page
    if (h.type == 2) {
      if (had_dict || seq >= (1u << 26)) { status = IX_FALLBACK; break; }
      had_dict = true;
    }
    if (h.type == 2 && ch.dict_off >= 0 && ch.dict_off != off) {  // seek to the data pages (:220-226)
      if (ch.data_off < 0) { status = IX_FALLBACK; break; }
      count += ch.data_off - off;
      off = ch.data_off;
    }
    seq++;
    if ((seq & 63) == 0) {
      if (!flush(64)) { status = IX_FALLBACK; break; }
      flushed = seq;
    }
  }
  if (status == IX_OK && seq > flushed && !flush(seq - flushed)) status = IX_FALLBACK;
  if (lane == 0) gp(res_in)[c] = make_uint4(status, status == IX_OK ? seq : 0u, seq, gen);
}

// ---------------------------------------------------------------------------
// CRC32 (IEEE) of every page block with a checksum
// ---------------------------------------------------------------------------
DEV uint32_t gf2_mulmod(uint32_t a, uint32_t b) {  // a·b mod P, reflected (zlib multmodp)
  uint32_t p = 0;
  for (uint32_t m = 1u << 31; m; m >>= 1) {
    if (a & m) p ^= b;
    b = (b & 1) ? (b >> 1) ^ kCrcPoly : b >> 1;
  }
  return p;
}
struct X2n { uint32_t v[32]; };
constexpr uint32_t x2n_mul(uint32_t a, uint32_t b) {
  uint32_t p = 0;
  for (uint32_t m = 1u << 31; m; m >>= 1) {
    if (a & m) p ^= b;
    b = (b & 1) ? (b >> 1) ^ kCrcPoly : b >> 1;
  }
  return p;
}
constexpr X2n make_x2n() {
  X2n t{};
  uint32_t p = 1u << 30;  // x^1
  t.v[0] = p;
  for (int n = 1; n < 32; n++) t.v[n] = p = x2n_mul(p, p);
  return t;
}
__constant__ X2n kX2n = make_x2n();  // x^(2^k) mod P

DEV uint32_t x8n_modp(uint64_t n) {  // x^(8n) mod P
  uint32_t p = 1u << 31;  // x^0
  for (uint32_t k = 3; n; n >>= 1, k++)
    if (n & 1) p = gf2_mulmod(kX2n.v[k & 31], p);
  return p;
}

constexpr uint32_t kCrcThreads = 256;

__global__ void __launch_bounds__(kCrcThreads) k_page_crc(const uint8_t *buf_in, int64_t len, int64_t file_off,
                                                          PageIxEntry *table_in, const uint32_t *table_n_in,
                                                          uint32_t table_cap) {
  __shared__ uint32_t T[4][256];
  __shared__ uint32_t wred[kCrcThreads / 64];
  const uint8_t *buf = gp(buf_in);
  PageIxEntry *table = gp(table_in);
  const uint32_t tid = threadIdx.x;
  {  // slicing-by-4 tables
    uint32_t c = tid;
    for (int k = 0; k < 8; k++) c = (c & 1) ? (c >> 1) ^ kCrcPoly : c >> 1;
    T[0][tid] = c;
  }
  wg_barrier();
  for (int j = 1; j < 4; j++) {
    const uint32_t c = T[j - 1][tid];
    T[j][tid] = (c >> 8) ^ T[0][c & 0xff];
    wg_barrier();
  }
  // An overflowing walk (count > capacity) left reserved slots unwritten: the host reruns it with a
  // larger table or keeps no entries, so no block of this table is checksummed. Otherwise every
  // slot below the count was written by the walk.
  const uint32_t n_entries = *gp(table_n_in);
  if (n_entries > table_cap) return;
  for (uint32_t e = blockIdx.x; e < n_entries; e += gridDim.x) {
    const PageIxEntry &h = table[e];
    const uint32_t fl = h.flags;
    if (!(fl & IXF_CRC)) continue;  // workgroup-uniform
    const int64_t L = h.csize;
    const int64_t b0 = h.hdr_off + h.hdr_len - file_off;  // block start (buffer-relative)
    const int64_t seg = ((L + kCrcThreads - 1) / kCrcThreads + 3) & ~(int64_t)3;
    const int64_t s0 = min(L, (int64_t)tid * seg), s1 = min(L, s0 + seg);
    uint32_t crc = 0xffffffffu;
    int64_t i = s0;
    // bytes up to a 4-aligned buffer position, then dwords, then the tail
    for (; i < s1 && ((b0 + i) & 3); i++) crc = T[0][(crc ^ buf[b0 + i]) & 0xff] ^ (crc >> 8);
    for (; i + 4 <= s1; i += 4) {
      crc ^= *(const uint32_t *)(buf + b0 + i);
      crc = T[3][crc & 0xff] ^ T[2][(crc >> 8) & 0xff] ^ T[1][(crc >> 16) & 0xff] ^ T[0][crc >> 24];
    }
    for (; i < s1; i++) crc = T[0][(crc ^ buf[b0 + i]) & 0xff] ^ (crc >> 8);
    crc = ~crc;
    // crc32(A || B) = x^(8|B|)·crc32(A) xor crc32(B): this segment's share of the block's checksum
    uint32_t part = (s1 > s0 && crc) ? (s1 == L ? crc : gf2_mulmod(x8n_modp((uint64_t)(L - s1)), crc)) : 0u;
    for (uint32_t o = 32; o; o >>= 1) part ^= __shfl_xor(part, o);
    if (lane_id() == 0) wred[tid >> 6] = part;
    wg_barrier();
    if (tid == 0) {
      uint32_t tot = 0;
      for (uint32_t w = 0; w < kCrcThreads / 64; w++) tot ^= wred[w];
      table[e].flags = fl | IXF_CRC_CHECKED | (tot == (uint32_t)h.crc ? IXF_CRC_OK : 0u);
    }
    wg_barrier();
  }
}

// ---------------------------------------------------------------------------
// Page bodies into the batch's page region
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_page_gather(const GatherJob *jobs_in, uint32_t njobs) {
  const GatherJob *jobs = gp(jobs_in);
  for (uint32_t j = blockIdx.x; j < njobs; j += gridDim.x) {
    const GatherJob g = jobs[j];
    uint8_t *dst = gp_u64<uint8_t>(g.dst);
    const uint8_t *src = gp_u64<const uint8_t>(g.src);
    // copy_bytes reads whole aligned 16-B source blocks (up to 16 bytes past its range): the last
    // 32 bytes of the block are copied bytewise so nothing past the resident bytes is read
    const uint64_t bulk = g.len > 32 ? g.len - 32 : 0;
    copy_bytes(dst, src, bulk, threadIdx.x, blockDim.x);
    for (uint64_t k = bulk + threadIdx.x; k < g.len; k += blockDim.x) dst[k] = src[k];
    if (threadIdx.x < 64) dst[g.len + threadIdx.x] = 0;
  }
}

// Before the walk: the entry counter to zero, every chunk's result to IX_FALLBACK (a chunk whose
// walk never reports stays with the host)
__global__ void __launch_bounds__(256) k_page_walk_init(uint32_t *table_n, uint4 *res, uint32_t nchunks) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t == 0) *gp(table_n) = 0;
  if (t < nchunks) gp(res)[t] = make_uint4(IX_FALLBACK, 0u, 0u, 0u);
}

hipError_t launch_page_walk(const uint8_t *buf, int64_t len, int64_t file_off, const PageIxChunk *chunks,
                            uint32_t nchunks, uint4 *res, PageIxEntry *table, uint32_t *table_n, uint32_t table_cap,
                            int validate_crc, uint32_t gen, hipStream_t s) {
  if (!nchunks) return hipSuccess;
#ifdef PQ_DIAG_STAMPS
  // diagnostic build only (tests/test_page_index.py): one chunk's table stores are dropped
  const char *skip_env = getenv("PQ_IX_TEST_SKIP_STORE");
  const uint32_t test_skip = skip_env ? (uint32_t)atoi(skip_env) : 0xffffffffu;
#else
  const uint32_t test_skip = 0xffffffffu;
#endif
  hipLaunchKernelGGL(k_page_walk_init, dim3((nchunks + 255) / 256), dim3(256), 0, s, table_n, res, nchunks);
  for (uint32_t c0 = 0; c0 < nchunks; c0 += kIxArgChunks) {
    const uint32_t n = std::min<uint32_t>(kIxArgChunks, nchunks - c0);
    IxChunkArgs a;
    memset(&a, 0, sizeof(a));
    memcpy(a.c, chunks + c0, n * sizeof(PageIxChunk));
    hipLaunchKernelGGL(k_page_walk, dim3(n), dim3(64), 0, s, buf, len, file_off, a, c0, res, table, table_n, table_cap, gen, test_skip);
  }
  if (validate_crc)
    hipLaunchKernelGGL(k_page_crc, dim3(2048), dim3(kCrcThreads), 0, s, buf, len, file_off, table,
                       (const uint32_t *)table_n, table_cap);
  return hipGetLastError();
}

hipError_t launch_page_gather(const GatherJob *jobs, uint32_t njobs, hipStream_t s) {
  if (!njobs) return hipSuccess;
  hipLaunchKernelGGL(k_page_gather, dim3(std::min<uint32_t>(njobs, 4096)), dim3(256), 0, s, jobs, njobs);
  return hipGetLastError();
}

}  // namespace pq
