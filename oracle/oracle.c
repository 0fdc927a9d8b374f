/*
 * oracle.c — CPU restatement of the fraugster/parquet-go (v0.12.0 line)
 * column-chunk read path. TEST INFRASTRUCTURE ONLY (see oracle.h): this is
 * the parity checker for libpqgpu, never part of the product path.
 *
 * Scope: FileReader open (file_meta.go:24-74, schema.go:893-1079),
 * readChunk/readPages (chunk_reader.go:182-362), page readers V1/V2
 * (page_v1.go:33-122, page_v2.go:31-131), dictionary page
 * (page_dict.go:35-72), value decoders (type_*.go), hybrid RLE/bit-packing
 * (hybrid_decoder.go:29-165), DELTA_BINARY_PACKED (deltabp_decoder.go),
 * block decompression (compress.go:34-123). Go I/O semantics
 * (bytes.Reader.Read, io.ReadFull, binary.ReadUvarint as of Go 1.17, the
 * toolchain pinned by the reference CI .circleci/config.yml) are restated
 * in the br_* helpers because the reference's error behaviour depends on
 * them.
 *
 * Third-party algorithms on the path and how they are pinned:
 *   golang/snappy v0.0.1 (vendored; go.mod pins v0.0.4) Decode —
 *     restated from the snappy block-format spec; parity unpinned beyond
 *     pyarrow's snappy codec round trips.
 *   compress/gzip (Go stdlib) — zlib inflate (gzip wrapper, multistream);
 *     parity unpinned beyond pyarrow's gzip codec round trips.
 *   apache/thrift compact protocol (vendored v0.15.0) — restated from the
 *     compact-protocol spec; pinned by pyarrow-written footers/headers.
 */
#include "oracle.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <zlib.h>

#define MAXI32 2147483647LL

/* ------------------------------------------------------------------ */
/* Go I/O semantics over an in-memory slice (bytes.Reader)             */
/* ------------------------------------------------------------------ */
typedef struct {
  const uint8_t *s;
  int64_t n; /* length */
  int64_t i; /* read position */
} breader;

static void br_init(breader *r, const uint8_t *s, int64_t n) { r->s = s; r->n = n < 0 ? 0 : n; r->i = 0; }
static int64_t br_rem(const breader *r) { return r->i >= r->n ? 0 : r->n - r->i; }

/* bytes.Reader.Read: EOF when exhausted (even for len(b)==0), else copies min. */
static int br_read(breader *r, uint8_t *b, int64_t len, int64_t *nread) {
  if (r->i >= r->n) { *nread = 0; return OR_ERR_EOF; }
  int64_t k = r->n - r->i;
  if (k > len) k = len;
  if (b && k) memcpy(b, r->s + r->i, (size_t)k);
  r->i += k;
  *nread = k;
  return OR_OK;
}

/* io.ReadFull: 0 bytes wanted -> ok; nothing read -> EOF; short -> ErrUnexpectedEOF. */
static int br_readfull(breader *r, uint8_t *b, int64_t len) {
  if (len <= 0) return OR_OK;
  int64_t got = 0;
  int e = br_read(r, b, len, &got);
  if (e) return e;
  if (got < len) return OR_ERR_UNEXPECTED_EOF;
  return OR_OK;
}

/* binary.ReadUvarint, Go 1.17 (EOF mid-varint returns io.EOF; overflow error). */
static int br_uvarint(breader *r, uint64_t *out) {
  uint64_t x = 0;
  unsigned s = 0;
  for (int i = 0;; i++) {
    if (r->i >= r->n) { *out = x; return OR_ERR_EOF; }
    uint8_t b = r->s[r->i++];
    if (b < 0x80) {
      if (i > 9 || (i == 9 && b > 1)) { *out = x; return OR_ERR_RANGE; }
      if (s < 64) x |= (uint64_t)b << s;
      *out = x;
      return OR_OK;
    }
    if (s < 64) x |= (uint64_t)(b & 0x7f) << s;
    s += 7;
  }
}

/* readUVariant32 helpers.go:165-182 */
static int read_uvariant32(breader *r, int32_t *out) {
  uint64_t v;
  int e = br_uvarint(r, &v);
  if (e) return e;
  if (v > (uint64_t)MAXI32) return OR_ERR_RANGE;
  *out = (int32_t)v;
  return OR_OK;
}

/* binary.ReadVarint (zigzag) */
static int br_varint(breader *r, int64_t *out) {
  uint64_t ux;
  int e = br_uvarint(r, &ux);
  int64_t x = (int64_t)(ux >> 1);
  if (ux & 1) x = ~x;
  *out = x;
  return e;
}

/* readVariant32 helpers.go:184-201 */
static int read_variant32(breader *r, int32_t *out) {
  int64_t v;
  int e = br_varint(r, &v);
  if (e) return e;
  if (v > MAXI32 || v < -MAXI32 - 1) return OR_ERR_RANGE;
  *out = (int32_t)v;
  return OR_OK;
}

/* readVariant64 helpers.go:210-217 */
static int read_variant64(breader *r, int64_t *out) { return br_varint(r, out); }

/* ------------------------------------------------------------------ */
/* Bit unpacking: unpack8int32_{bw} / unpack8int64_{bw}                */
/* (bitbacking32.go:10-44, bitpacking64.go:10; generator semantics     */
/* bitpack_gen.go:19-59: LSB-first bits within little-endian bytes)    */
/* ------------------------------------------------------------------ */
void or_unpack8_int64(const uint8_t *data, int bw, int64_t out[8]) {
  for (int i = 0; i < 8; i++) {
    uint64_t v = 0;
    for (int b = 0; b < bw; b++) {
      int bit = i * bw + b;
      if ((data[bit >> 3] >> (bit & 7)) & 1) v |= (uint64_t)1 << b;
    }
    out[i] = (int64_t)v;
  }
}

void or_unpack8_int32(const uint8_t *data, int bw, int32_t out[8]) {
  int64_t t[8];
  or_unpack8_int64(data, bw, t);
  for (int i = 0; i < 8; i++) out[i] = (int32_t)(uint32_t)(uint64_t)t[i];
}

/* ------------------------------------------------------------------ */
/* hybridDecoder  hybrid_decoder.go:29-165                             */
/* ------------------------------------------------------------------ */
typedef struct {
  breader r;
  int has_r;
  int bw;
  int rle_size;
  int32_t bp[8];
  uint32_t rle_count;
  int32_t rle_value;
  uint32_t bp_count;
  uint8_t bp_pos;
} hybrid;

static void hyb_new(hybrid *h, int bw) { /* newHybridDecoder :47-54 */
  memset(h, 0, sizeof(*h));
  h->bw = bw;
  h->rle_size = (bw + 7) / 8;
}

static void hyb_init(hybrid *h, const uint8_t *s, int64_t n) { br_init(&h->r, s, n); h->has_r = 1; }

/* readRLERunValue :115-130 (value >= 2^bw -> error) */
static int hyb_read_rle_value(hybrid *h) {
  uint8_t v[4] = {0, 0, 0, 0};
  int64_t n;
  int e = br_read(&h->r, v, h->rle_size, &n);
  if (e) return e;
  if (n != h->rle_size) return OR_ERR_UNEXPECTED_EOF;
  uint32_t x = (uint32_t)v[0] | ((uint32_t)v[1] << 8) | ((uint32_t)v[2] << 16) | ((uint32_t)v[3] << 24);
  h->rle_value = (int32_t)x;
  if (h->bw < 32 && (x >> h->bw) != 0) return OR_ERR_INVALID; /* "rle: RLE run value is too large" */
  return OR_OK;
}

/* readBitPackedRun :132-140 — bare Read: a short final group is zero-filled (Q3) */
static int hyb_read_bp_run(hybrid *h) {
  uint8_t data[32];
  memset(data, 0, sizeof(data));
  int64_t n;
  int e = br_read(&h->r, data, h->bw, &n);
  if (e) return e;
  or_unpack8_int32(data, h->bw, h->bp);
  return OR_OK;
}

/* readRunHeader :142-165 */
static int hyb_read_header(hybrid *h) {
  int32_t hd;
  int e = read_uvariant32(&h->r, &hd);
  if (e) return e;
  if (hd & 1) {
    h->bp_count = (uint32_t)(hd >> 1);
    if (h->bp_count == 0) return OR_ERR_INVALID; /* "rle: empty bit-packed run" */
    h->bp_pos = 0;
  } else {
    h->rle_count = (uint32_t)(hd >> 1);
    if (h->rle_count == 0) return OR_ERR_INVALID; /* "rle: empty RLE run" */
    return hyb_read_rle_value(h);
  }
  return OR_OK;
}

/* next :81-113 */
static int hyb_next(hybrid *h, int32_t *out) {
  if (h->bw == 0) { *out = 0; return OR_OK; }
  if (!h->has_r) return OR_ERR_INVALID; /* "reader is not initialized" */
  int e;
  if (h->rle_count == 0 && h->bp_count == 0 && h->bp_pos == 0) {
    if ((e = hyb_read_header(h))) return e;
  }
  if (h->rle_count > 0) {
    *out = h->rle_value;
    h->rle_count--;
  } else if (h->bp_count > 0 || h->bp_pos > 0) {
    if (h->bp_pos == 0) {
      if ((e = hyb_read_bp_run(h))) return e;
      h->bp_count--;
    }
    *out = h->bp[h->bp_pos];
    h->bp_pos = (uint8_t)((h->bp_pos + 1) % 8);
  } else {
    return OR_ERR_EOF;
  }
  return OR_OK;
}

int or_hybrid_decode(const uint8_t *buf, size_t len, int bw, int64_t n, int32_t *out, int64_t *decoded) {
  hybrid h;
  hyb_new(&h, bw);
  hyb_init(&h, buf, (int64_t)len);
  for (int64_t i = 0; i < n; i++) {
    int e = hyb_next(&h, &out[i]);
    if (e) { *decoded = i; return e; }
  }
  *decoded = n;
  return OR_OK;
}

/* ------------------------------------------------------------------ */
/* deltaBitPackDecoder32/64  deltabp_decoder.go:13-333                 */
/* One implementation parameterised on the value width (64 or 32);     */
/* 32-bit arithmetic wraps exactly like Go int32.                      */
/* ------------------------------------------------------------------ */
typedef struct {
  breader *r;
  int is64;
  int32_t block_size, mb_count, values_count, mb_value_count;
  int64_t prev, min_delta;
  uint8_t widths[256];
  uint8_t *widths_dyn;
  int32_t cur_mb;
  uint8_t cur_w;
  int32_t mb_pos, position;
  int64_t mb_vals[8];
} delta;

static uint8_t *dl_widths(delta *d) { return d->widths_dyn ? d->widths_dyn : d->widths; }

/* readBlockHeader :51-86 / :210-245 */
static int dl_read_block_header(delta *d) {
  int e;
  if ((e = read_uvariant32(d->r, &d->block_size))) return e;
  if (d->block_size <= 0 && d->block_size % 128 != 0) return OR_ERR_INVALID; /* Q8: never true */
  if ((e = read_uvariant32(d->r, &d->mb_count))) return e;
  if (d->mb_count <= 0 || d->block_size % d->mb_count != 0) return OR_ERR_INVALID;
  d->mb_value_count = d->block_size / d->mb_count;
  if (d->mb_value_count == 0) return OR_ERR_INVALID;
  if ((e = read_uvariant32(d->r, &d->values_count))) return e;
  if (d->values_count < 0) return OR_ERR_INVALID;
  if (d->is64) {
    if ((e = read_variant64(d->r, &d->prev))) return e;
  } else {
    int32_t v;
    if ((e = read_variant32(d->r, &v))) return e;
    d->prev = v;
  }
  return OR_OK;
}

/* readMiniBlockHeader :88-111 / :247-270 */
static int dl_read_mb_header(delta *d) {
  int e;
  if (d->is64) {
    if ((e = read_variant64(d->r, &d->min_delta))) return e;
  } else {
    int32_t v;
    if ((e = read_variant32(d->r, &v))) return e;
    d->min_delta = v;
  }
  if (!d->widths_dyn && d->mb_count > 256) {
    d->widths_dyn = (uint8_t *)malloc((size_t)d->mb_count);
    if (!d->widths_dyn) return OR_ERR_NOMEM;
  }
  uint8_t *w = dl_widths(d);
  if ((e = br_readfull(d->r, w, d->mb_count))) return e;
  for (int32_t i = 0; i < d->mb_count; i++)
    if (w[i] > (d->is64 ? 64 : 32)) return OR_ERR_INVALID;
  d->cur_mb = 0;
  return OR_OK;
}

/* init :35-49 */
static int dl_init(delta *d, breader *r, int is64) {
  memset(d, 0, sizeof(*d));
  d->r = r;
  d->is64 = is64;
  int e;
  if ((e = dl_read_block_header(d))) return e;
  return dl_read_mb_header(d);
}

static void dl_free(delta *d) { free(d->widths_dyn); d->widths_dyn = NULL; }

/* next :113-174 / :272-333 (look-ahead Q1, padding skip Q2) */
static int dl_next(delta *d, int64_t *out) {
  int e;
  if (d->position >= d->values_count) return OR_ERR_EOF;
  if (d->position % 8 == 0) {
    if (d->position % d->mb_value_count == 0) {
      if (d->cur_mb >= d->mb_count) {
        if ((e = dl_read_mb_header(d))) return e;
      }
      d->cur_w = dl_widths(d)[d->cur_mb];
      d->mb_pos = 0;
      d->cur_mb++;
    }
    int32_t w = d->cur_w;
    uint8_t buf[64];
    memset(buf, 0, sizeof(buf));
    if ((e = br_readfull(d->r, buf, w))) return e;
    if (d->is64) {
      or_unpack8_int64(buf, w, d->mb_vals);
    } else {
      int32_t t[8];
      or_unpack8_int32(buf, w, t);
      for (int i = 0; i < 8; i++) d->mb_vals[i] = t[i];
    }
    d->mb_pos += w;
    if ((int64_t)d->position + 8 >= d->values_count) {
      int64_t l = (int64_t)(d->mb_value_count / 8) * w - d->mb_pos;
      if (l < 0) return OR_ERR_INVALID; /* "invalid stream" */
      {
        int64_t skip = l, avail = br_rem(d->r);
        d->r->i += skip < avail ? skip : avail; /* ReadFull, error ignored */
      }
      for (int32_t i = d->cur_mb; i < d->mb_count; i++) {
        int32_t w2 = dl_widths(d)[d->cur_mb]; /* sic: indexes cur_mb, not i (Q2) */
        if (w2 != 0) {
          int64_t skip = (int64_t)(d->mb_value_count / 8) * w2, avail = br_rem(d->r);
          d->r->i += skip < avail ? skip : avail;
        }
      }
    }
  }
  int64_t ret = d->prev;
  if (d->is64) {
    d->prev = (int64_t)((uint64_t)d->prev + (uint64_t)d->mb_vals[d->position % 8] + (uint64_t)d->min_delta);
  } else {
    uint32_t p = (uint32_t)(int32_t)d->prev + (uint32_t)(int32_t)d->mb_vals[d->position % 8] +
                 (uint32_t)(int32_t)d->min_delta;
    d->prev = (int32_t)p;
  }
  d->position++;
  *out = ret;
  return OR_OK;
}

int or_delta_decode64(const uint8_t *buf, size_t len, int64_t n, int64_t *out, int64_t *decoded) {
  breader r;
  br_init(&r, buf, (int64_t)len);
  delta d;
  int e = dl_init(&d, &r, 1);
  *decoded = 0;
  if (e) { dl_free(&d); return e; }
  for (int64_t i = 0; i < n; i++) {
    e = dl_next(&d, &out[i]);
    if (e) { *decoded = i; dl_free(&d); return e; }
  }
  *decoded = n;
  dl_free(&d);
  return OR_OK;
}

int or_delta_decode32(const uint8_t *buf, size_t len, int64_t n, int32_t *out, int64_t *decoded) {
  breader r;
  br_init(&r, buf, (int64_t)len);
  delta d;
  int e = dl_init(&d, &r, 0);
  *decoded = 0;
  if (e) { dl_free(&d); return e; }
  for (int64_t i = 0; i < n; i++) {
    int64_t v;
    e = dl_next(&d, &v);
    if (e) { *decoded = i; dl_free(&d); return e; }
    out[i] = (int32_t)v;
  }
  *decoded = n;
  dl_free(&d);
  return OR_OK;
}

/* ------------------------------------------------------------------ */
/* Thrift compact protocol (apache/thrift v0.15.0 TCompactProtocol)    */
/* ------------------------------------------------------------------ */
enum { CT_STOP = 0, CT_TRUE = 1, CT_FALSE = 2, CT_BYTE = 3, CT_I16 = 4, CT_I32 = 5, CT_I64 = 6,
       CT_DOUBLE = 7, CT_BINARY = 8, CT_LIST = 9, CT_SET = 10, CT_MAP = 11, CT_STRUCT = 12 };

typedef struct {
  breader *r;
  int err;
} tc;

static int tc_byte(tc *t, uint8_t *b) {
  if (t->err) return t->err;
  if (t->r->i >= t->r->n) return t->err = OR_ERR_THRIFT;
  *b = t->r->s[t->r->i++];
  return OR_OK;
}

static uint64_t tc_uvar(tc *t) { /* readVarint64: no overflow check */
  uint64_t x = 0;
  unsigned s = 0;
  for (;;) {
    uint8_t b;
    if (tc_byte(t, &b)) return 0;
    if (s < 64) x |= (uint64_t)(b & 0x7f) << s;
    if (!(b & 0x80)) break;
    s += 7;
  }
  return x;
}
static int64_t tc_zz64(tc *t) { uint64_t u = tc_uvar(t); return (int64_t)(u >> 1) ^ -(int64_t)(u & 1); }
static int32_t tc_zz32(tc *t) { uint32_t u = (uint32_t)tc_uvar(t); return (int32_t)(u >> 1) ^ -(int32_t)(u & 1); }

static void tc_skip(tc *t, int type, int depth);

static void tc_skip_binary(tc *t) {
  int32_t len = (int32_t)tc_uvar(t);
  if (t->err) return;
  if (len < 0 || (int64_t)len > br_rem(t->r)) { t->err = OR_ERR_THRIFT; return; }
  t->r->i += len;
}

static int tc_list_begin(tc *t, int *etype, int32_t *size) {
  uint8_t b;
  if (tc_byte(t, &b)) return t->err;
  int32_t sz = (b >> 4) & 0x0f;
  if (sz == 15) sz = (int32_t)tc_uvar(t);
  if (t->err) return t->err;
  if (sz < 0) return t->err = OR_ERR_THRIFT;
  if ((b & 0x0f) > CT_STRUCT) return t->err = OR_ERR_THRIFT; /* getTType: unknown compact type */
  *etype = b & 0x0f;
  *size = sz;
  return OR_OK;
}

static void tc_skip(tc *t, int type, int depth) {
  if (t->err) return;
  if (depth > 64) { t->err = OR_ERR_THRIFT; return; }
  uint8_t b;
  switch (type) {
    case CT_TRUE: case CT_FALSE: tc_byte(t, &b); break; /* bool inside collections */
    case CT_BYTE: tc_byte(t, &b); break;
    case CT_I16: case CT_I32: case CT_I64: tc_uvar(t); break;
    case CT_DOUBLE:
      if (br_rem(t->r) < 8) t->err = OR_ERR_THRIFT; else t->r->i += 8;
      break;
    case CT_BINARY: tc_skip_binary(t); break;
    case CT_LIST: case CT_SET: {
      int et; int32_t n;
      if (tc_list_begin(t, &et, &n)) return;
      for (int32_t i = 0; i < n && !t->err; i++) tc_skip(t, et, depth + 1);
      break;
    }
    case CT_MAP: {
      int32_t n = (int32_t)tc_uvar(t);
      if (t->err) return;
      if (n < 0) { t->err = OR_ERR_THRIFT; return; }
      if (n == 0) break;
      if (tc_byte(t, &b)) return;
      for (int32_t i = 0; i < n && !t->err; i++) { tc_skip(t, b >> 4, depth + 1); tc_skip(t, b & 0x0f, depth + 1); }
      break;
    }
    case CT_STRUCT: {
      int16_t last = 0;
      for (;;) {
        if (tc_byte(t, &b)) return;
        if ((b & 0x0f) == CT_STOP) break;
        int ty = b & 0x0f;
        int mod = b >> 4;
        int16_t id = mod ? (int16_t)(last + mod) : (int16_t)tc_zz32(t);
        last = id;
        if (ty != CT_TRUE && ty != CT_FALSE) tc_skip(t, ty, depth + 1);
        if (ty > CT_STRUCT) { t->err = OR_ERR_THRIFT; return; }
      }
      break;
    }
    default: t->err = OR_ERR_THRIFT;
  }
}

/* Field iteration: returns 0 at STOP or error; sets *id, *type. */
typedef struct { int16_t last; } tc_struct;
static int tc_field(tc *t, tc_struct *st, int16_t *id, int *type) {
  uint8_t b;
  if (tc_byte(t, &b)) return 0;
  if ((b & 0x0f) == CT_STOP) return 0;
  int mod = b >> 4;
  *id = mod ? (int16_t)(st->last + mod) : (int16_t)tc_zz32(t);
  if (t->err) return 0;
  st->last = *id;
  *type = b & 0x0f;
  if (*type > CT_STRUCT) { t->err = OR_ERR_THRIFT; return 0; }
  return 1;
}
static int64_t tc_int(tc *t, int ty) {
  if (ty == CT_BYTE) { uint8_t b = 0; tc_byte(t, &b); return (int8_t)b; }
  return ty == CT_I64 ? tc_zz64(t) : (int64_t)tc_zz32(t);
}
static void tc_skip_field(tc *t, int ty) { if (ty != CT_TRUE && ty != CT_FALSE) tc_skip(t, ty, 1); }

/* ---- Parquet thrift structs (parquet/parquet.thrift) ---- */
typedef struct {
  int set_num_values, set_encoding, set_def, set_rep;
  int32_t num_values, encoding, def_enc, rep_enc;
} dph_t;
typedef struct { int set_num_values, set_encoding; int32_t num_values, encoding; } dict_ph_t;
typedef struct {
  int set_nv, set_nn, set_nr, set_enc, set_dl, set_rl;
  int32_t num_values, num_nulls, num_rows, encoding, def_len, rep_len;
  int is_compressed;
} dph2_t;
typedef struct {
  int set_type, set_usize, set_csize;
  int32_t type, usize, csize;
  int has_crc;
  int32_t crc;
  int has_dph, has_dict, has_dph2;
  dph_t dph;
  dict_ph_t dict;
  dph2_t dph2;
} page_header_t;

static void rd_dph(tc *t, dph_t *h) {
  tc_struct st = {0}; int16_t id; int ty;
  while (tc_field(t, &st, &id, &ty)) {
    if (id == 1 && ty == CT_I32) { h->num_values = (int32_t)tc_int(t, ty); h->set_num_values = 1; }
    else if (id == 2 && ty == CT_I32) { h->encoding = (int32_t)tc_int(t, ty); h->set_encoding = 1; }
    else if (id == 3 && ty == CT_I32) { h->def_enc = (int32_t)tc_int(t, ty); h->set_def = 1; }
    else if (id == 4 && ty == CT_I32) { h->rep_enc = (int32_t)tc_int(t, ty); h->set_rep = 1; }
    else tc_skip_field(t, ty);
  }
  if (!t->err && !(h->set_num_values && h->set_encoding && h->set_def && h->set_rep)) t->err = OR_ERR_THRIFT;
}
static void rd_dict(tc *t, dict_ph_t *h) {
  tc_struct st = {0}; int16_t id; int ty;
  while (tc_field(t, &st, &id, &ty)) {
    if (id == 1 && ty == CT_I32) { h->num_values = (int32_t)tc_int(t, ty); h->set_num_values = 1; }
    else if (id == 2 && ty == CT_I32) { h->encoding = (int32_t)tc_int(t, ty); h->set_encoding = 1; }
    else tc_skip_field(t, ty);
  }
  if (!t->err && !(h->set_num_values && h->set_encoding)) t->err = OR_ERR_THRIFT;
}
static void rd_dph2(tc *t, dph2_t *h) {
  tc_struct st = {0}; int16_t id; int ty;
  h->is_compressed = 1;
  while (tc_field(t, &st, &id, &ty)) {
    if (ty == CT_I32 && id >= 1 && id <= 6) {
      int32_t v = (int32_t)tc_int(t, ty);
      switch (id) {
        case 1: h->num_values = v; h->set_nv = 1; break;
        case 2: h->num_nulls = v; h->set_nn = 1; break;
        case 3: h->num_rows = v; h->set_nr = 1; break;
        case 4: h->encoding = v; h->set_enc = 1; break;
        case 5: h->def_len = v; h->set_dl = 1; break;
        case 6: h->rep_len = v; h->set_rl = 1; break;
      }
    } else if (id == 7 && (ty == CT_TRUE || ty == CT_FALSE)) {
      h->is_compressed = ty == CT_TRUE;
    } else tc_skip_field(t, ty);
  }
  if (!t->err && !(h->set_nv && h->set_nn && h->set_nr && h->set_enc && h->set_dl && h->set_rl)) t->err = OR_ERR_THRIFT;
}
static int rd_page_header(breader *r, page_header_t *h) {
  memset(h, 0, sizeof(*h));
  tc t = {r, 0};
  tc_struct st = {0}; int16_t id; int ty;
  while (tc_field(&t, &st, &id, &ty)) {
    if (id == 1 && ty == CT_I32) { h->type = (int32_t)tc_int(&t, ty); h->set_type = 1; }
    else if (id == 2 && ty == CT_I32) { h->usize = (int32_t)tc_int(&t, ty); h->set_usize = 1; }
    else if (id == 3 && ty == CT_I32) { h->csize = (int32_t)tc_int(&t, ty); h->set_csize = 1; }
    else if (id == 4 && ty == CT_I32) { h->crc = (int32_t)tc_int(&t, ty); h->has_crc = 1; }
    else if (id == 5 && ty == CT_STRUCT) { h->has_dph = 1; rd_dph(&t, &h->dph); }
    else if (id == 7 && ty == CT_STRUCT) { h->has_dict = 1; rd_dict(&t, &h->dict); }
    else if (id == 8 && ty == CT_STRUCT) { h->has_dph2 = 1; rd_dph2(&t, &h->dph2); }
    else tc_skip_field(&t, ty);
  }
  if (!t.err && !(h->set_type && h->set_usize && h->set_csize)) t.err = OR_ERR_THRIFT;
  return t.err;
}

/* FileMetaData subset */
typedef struct {
  int has_type; int32_t type;
  int has_type_length; int32_t type_length;
  int has_rep; int32_t rep;
  char name[128];
  int has_name;
  int has_num_children; int32_t num_children;
} schema_el;

typedef struct {
  int has_meta;
  int has_file_path;
  int32_t type;
  int32_t codec;
  int64_t num_values, total_uncompressed, total_compressed, data_page_offset;
  int has_dict_offset;
  int64_t dict_offset;
} col_chunk;

typedef struct {
  col_chunk *cols;
  int32_t ncols;
  int64_t num_rows;
} row_group;

typedef struct {
  int32_t physical_type, type_length, max_def, max_rep, rep;
  char path[256];
  int32_t path_len, node_rep[64];
} leaf_col;

struct or_file {
  const uint8_t *buf;
  int64_t len;
  schema_el *schema;
  int32_t nschema;
  row_group *rgs;
  int32_t nrgs;
  leaf_col *leaves;
  int32_t nleaves;
};

static void rd_schema_el(tc *t, schema_el *e) {
  tc_struct st = {0}; int16_t id; int ty;
  memset(e, 0, sizeof(*e));
  while (tc_field(t, &st, &id, &ty)) {
    if (id == 1 && ty == CT_I32) { e->type = (int32_t)tc_int(t, ty); e->has_type = 1; }
    else if (id == 2 && ty == CT_I32) { e->type_length = (int32_t)tc_int(t, ty); e->has_type_length = 1; }
    else if (id == 3 && ty == CT_I32) { e->rep = (int32_t)tc_int(t, ty); e->has_rep = 1; }
    else if (id == 4 && ty == CT_BINARY) {
      int32_t len = (int32_t)tc_uvar(t);
      if (t->err) return;
      if (len < 0 || (int64_t)len > br_rem(t->r)) { t->err = OR_ERR_THRIFT; return; }
      int32_t k = len < 127 ? len : 127;
      memcpy(e->name, t->r->s + t->r->i, (size_t)k);
      e->name[k] = 0;
      t->r->i += len;
      e->has_name = 1;
    } else if (id == 5 && ty == CT_I32) { e->num_children = (int32_t)tc_int(t, ty); e->has_num_children = 1; }
    else tc_skip_field(t, ty);
  }
  if (!t->err && !e->has_name) t->err = OR_ERR_THRIFT;
}

static void rd_col_meta(tc *t, col_chunk *c) {
  tc_struct st = {0}; int16_t id; int ty;
  int set_type = 0, set_enc = 0, set_path = 0, set_codec = 0, set_nv = 0, set_tu = 0, set_tc = 0, set_dpo = 0;
  while (tc_field(t, &st, &id, &ty)) {
    if (id == 1 && ty == CT_I32) { c->type = (int32_t)tc_int(t, ty); set_type = 1; }
    else if (id == 2 && ty == CT_LIST) { set_enc = 1; tc_skip(t, ty, 1); }
    else if (id == 3 && ty == CT_LIST) { set_path = 1; tc_skip(t, ty, 1); }
    else if (id == 4 && ty == CT_I32) { c->codec = (int32_t)tc_int(t, ty); set_codec = 1; }
    else if (id == 5 && ty == CT_I64) { c->num_values = tc_int(t, ty); set_nv = 1; }
    else if (id == 6 && ty == CT_I64) { c->total_uncompressed = tc_int(t, ty); set_tu = 1; }
    else if (id == 7 && ty == CT_I64) { c->total_compressed = tc_int(t, ty); set_tc = 1; }
    else if (id == 9 && ty == CT_I64) { c->data_page_offset = tc_int(t, ty); set_dpo = 1; }
    else if (id == 11 && ty == CT_I64) { c->dict_offset = tc_int(t, ty); c->has_dict_offset = 1; }
    else tc_skip_field(t, ty);
  }
  if (!t->err && !(set_type && set_enc && set_path && set_codec && set_nv && set_tu && set_tc && set_dpo))
    t->err = OR_ERR_THRIFT;
}

static void rd_col_chunk(tc *t, col_chunk *c) {
  tc_struct st = {0}; int16_t id; int ty;
  int set_fo = 0;
  memset(c, 0, sizeof(*c));
  while (tc_field(t, &st, &id, &ty)) {
    if (id == 1 && ty == CT_BINARY) { c->has_file_path = 1; tc_skip(t, ty, 1); }
    else if (id == 2 && ty == CT_I64) { tc_int(t, ty); set_fo = 1; }
    else if (id == 3 && ty == CT_STRUCT) { c->has_meta = 1; rd_col_meta(t, c); }
    else tc_skip_field(t, ty);
  }
  if (!t->err && !set_fo) t->err = OR_ERR_THRIFT;
}

static void rd_row_group(tc *t, row_group *g) {
  tc_struct st = {0}; int16_t id; int ty;
  int set_cols = 0, set_tbs = 0, set_nr = 0;
  memset(g, 0, sizeof(*g));
  while (tc_field(t, &st, &id, &ty)) {
    if (id == 1 && ty == CT_LIST) {
      int et; int32_t n;
      /* parquet.go RowGroup.ReadField1: the list's element type is not checked, every element is
         read as a ColumnChunk struct */
      if (tc_list_begin(t, &et, &n)) return;
      if ((int64_t)n > br_rem(t->r)) { t->err = OR_ERR_THRIFT; return; }
      g->cols = (col_chunk *)calloc((size_t)(n ? n : 1), sizeof(col_chunk));
      if (!g->cols) { t->err = OR_ERR_NOMEM; return; }
      g->ncols = n;
      for (int32_t i = 0; i < n && !t->err; i++) rd_col_chunk(t, &g->cols[i]);
      set_cols = 1;
    } else if (id == 2 && ty == CT_I64) { tc_int(t, ty); set_tbs = 1; }
    else if (id == 3 && ty == CT_I64) { g->num_rows = tc_int(t, ty); set_nr = 1; }
    else tc_skip_field(t, ty);
  }
  if (!t->err && !(set_cols && set_tbs && set_nr)) t->err = OR_ERR_THRIFT;
}

static int rd_file_meta(breader *r, or_file *f) {
  tc t = {r, 0};
  tc_struct st = {0}; int16_t id; int ty;
  int set_ver = 0, set_schema = 0, set_nr = 0, set_rgs = 0;
  while (tc_field(&t, &st, &id, &ty)) {
    if (id == 1 && ty == CT_I32) { tc_int(&t, ty); set_ver = 1; }
    else if (id == 2 && ty == CT_LIST) {
      int et; int32_t n;
      /* FileMetaData.ReadField2: elements read as SchemaElement whatever the element type */
      if (tc_list_begin(&t, &et, &n)) break;
      if ((int64_t)n > br_rem(r)) { t.err = OR_ERR_THRIFT; break; }
      f->schema = (schema_el *)calloc((size_t)(n ? n : 1), sizeof(schema_el));
      if (!f->schema) return OR_ERR_NOMEM;
      f->nschema = n;
      for (int32_t i = 0; i < n && !t.err; i++) rd_schema_el(&t, &f->schema[i]);
      set_schema = 1;
    } else if (id == 3 && ty == CT_I64) { tc_int(&t, ty); set_nr = 1; }
    else if (id == 4 && ty == CT_LIST) {
      int et; int32_t n;
      /* FileMetaData.ReadField4: elements read as RowGroup whatever the element type */
      if (tc_list_begin(&t, &et, &n)) break;
      if ((int64_t)n > br_rem(r)) { t.err = OR_ERR_THRIFT; break; }
      f->rgs = (row_group *)calloc((size_t)(n ? n : 1), sizeof(row_group));
      if (!f->rgs) return OR_ERR_NOMEM;
      f->nrgs = n;
      for (int32_t i = 0; i < n && !t.err; i++) rd_row_group(&t, &f->rgs[i]);
      set_rgs = 1;
    } else tc_skip_field(&t, ty);
  }
  if (!t.err && !(set_ver && set_schema && set_nr && set_rgs)) t.err = OR_ERR_THRIFT;
  return t.err;
}

/* ------------------------------------------------------------------ */
/* Schema -> leaf columns  schema.go:893-1079                          */
/* ------------------------------------------------------------------ */
static int add_leaf(or_file *f, const char *path, schema_el *e, int d, int r, const int32_t *reps, int nreps) {
  leaf_col *nl = (leaf_col *)realloc(f->leaves, sizeof(leaf_col) * (size_t)(f->nleaves + 1));
  if (!nl) return OR_ERR_NOMEM;
  f->leaves = nl;
  leaf_col *c = &f->leaves[f->nleaves++];
  c->physical_type = e->type;
  c->type_length = e->has_type_length ? e->type_length : 0;
  c->max_def = d;
  c->max_rep = r;
  c->rep = e->rep;
  snprintf(c->path, sizeof(c->path), "%s", path);
  c->path_len = nreps < 63 ? nreps + 1 : 64;
  for (int k = 0; k < c->path_len - 1; k++) c->node_rep[k] = reps[k];
  c->node_rep[c->path_len - 1] = e->rep;
  /* getValuesStore data_store.go:325-362 */
  if (e->type < 0 || e->type > 7) return OR_ERR_UNSUPPORTED;
  if (e->type == 7 && !e->has_type_length) return OR_ERR_INVALID;
  return OR_OK;
}

/* readColumnSchema :893-924 */
static int read_column_schema(or_file *f, int32_t base, int32_t idx, const char *path, int d, int r, int32_t *next,
                              const int32_t *reps, int nreps) {
  schema_el *s = &f->schema[base + idx];
  if (!s->name[0]) return OR_ERR_INVALID;
  if (!s->has_rep) return OR_ERR_INVALID;
  if (s->rep != 0) d++;
  if (s->rep == 2) r++;
  char p[256];
  snprintf(p, sizeof(p), "%s%s%s", path, path[0] ? "." : "", s->name);
  int e = add_leaf(f, p, s, d, r, reps, nreps);
  if (e) return e;
  *next = idx + 1;
  return OR_OK;
}

/* readGroupSchema :926-990 */
static int read_group_schema(or_file *f, int32_t base, int32_t n, int32_t idx, const char *path, int d, int r,
                             int32_t *next, int depth, int32_t *reps) {
  if (depth > 1000) return OR_ERR_INVALID;
  if (n <= idx) return OR_ERR_INVALID;
  schema_el *s = &f->schema[base + idx];
  if (s->has_type) return OR_ERR_INVALID;
  if (!s->has_num_children) return OR_ERR_INVALID;
  if (s->num_children <= 0) return OR_ERR_INVALID;
  int32_t l = s->num_children;
  if ((int64_t)n <= (int64_t)idx + l) return OR_ERR_INVALID;
  if (s->has_rep && s->rep != 0) d++;
  if (s->has_rep && s->rep == 2) r++;
  if (depth < 63) reps[depth] = s->has_rep ? s->rep : 0;  /* this group's node on its children's paths */
  char p[256];
  snprintf(p, sizeof(p), "%s%s%s", path, path[0] ? "." : "", s->name);
  idx++;
  for (int32_t i = 0; i < l; i++) {
    if (n <= idx) return OR_ERR_INVALID;
    int e;
    if (!f->schema[base + idx].has_type) e = read_group_schema(f, base, n, idx, p, d, r, &idx, depth + 1, reps);
    else e = read_column_schema(f, base, idx, p, d, r, &idx, reps, depth + 1 < 63 ? depth + 1 : 63);
    if (e) return e;
  }
  *next = idx;
  return OR_OK;
}

/* makeSchema :1048-1079 + readSchema :992-1015 (schema[0] is the root) */
static int make_schema(or_file *f) {
  if (f->nschema < 1) return OR_ERR_INVALID;
  int32_t n = f->nschema - 1;
  int32_t reps[64];
  for (int32_t idx = 0; idx < n;) {
    int e;
    if (!f->schema[1 + idx].has_type) e = read_group_schema(f, 1, n, idx, "", 0, 0, &idx, 0, reps);
    else e = read_column_schema(f, 1, idx, "", 0, 0, &idx, reps, 0);
    if (e) return e;
  }
  return OR_OK;
}

static void file_free(or_file *f) {
  if (!f) return;
  free(f->schema);
  if (f->rgs)
    for (int32_t i = 0; i < f->nrgs; i++) free(f->rgs[i].cols);
  free(f->rgs);
  free(f->leaves);
  free(f);
}

/* NewFileReaderWithOptions file_reader.go:32-63 + ReadFileMetaDataWithContext file_meta.go:24-74 */
int or_file_open(const uint8_t *buf, size_t len, or_file **out, char *err, size_t errlen) {
  *out = NULL;
  if (err && errlen) err[0] = 0;
  int64_t n = (int64_t)len;
  if (n < 4 || memcmp(buf, "PAR1", 4) != 0) {
    if (err) snprintf(err, errlen, "invalid parquet file header");
    return n < 4 ? OR_ERR_EOF : OR_ERR_INVALID;
  }
  if (n < 8 || memcmp(buf + n - 4, "PAR1", 4) != 0) {
    if (err) snprintf(err, errlen, "invalid parquet file footer");
    return OR_ERR_INVALID;
  }
  int32_t fl;
  memcpy(&fl, buf + n - 8, 4);
  if (fl <= 0) {
    if (err) snprintf(err, errlen, "invalid footer len %d", fl);
    return OR_ERR_INVALID;
  }
  int64_t start = n - 8 - (int64_t)fl;
  if (start < 0) {
    if (err) snprintf(err, errlen, "seek file meta data failed");
    return OR_ERR_INVALID;
  }
  or_file *f = (or_file *)calloc(1, sizeof(or_file));
  if (!f) return OR_ERR_NOMEM;
  f->buf = buf;
  f->len = n;
  breader r;
  br_init(&r, buf + start, fl);
  int e = rd_file_meta(&r, f);
  if (e) {
    if (err) snprintf(err, errlen, "read file meta failed");
    file_free(f);
    return e;
  }
  e = make_schema(f);
  if (e) {
    if (err) snprintf(err, errlen, "creating schema failed");
    file_free(f);
    return e;
  }
  *out = f;
  return OR_OK;
}

void or_file_close(or_file *f) { file_free(f); }
int or_file_num_row_groups(const or_file *f) { return f->nrgs; }
int or_file_num_columns(const or_file *f) { return f->nleaves; }
int64_t or_file_row_group_num_rows(const or_file *f, int rg) {
  return (rg < 0 || rg >= f->nrgs) ? -1 : f->rgs[rg].num_rows;
}
int or_file_column_info(const or_file *f, int col, or_column_info *out) {
  if (col < 0 || col >= f->nleaves) return OR_ERR_ARG;
  const leaf_col *c = &f->leaves[col];
  out->physical_type = c->physical_type;
  out->type_length = c->type_length;
  out->max_def = c->max_def;
  out->max_rep = c->max_rep;
  out->repetition = c->rep;
  snprintf(out->path, sizeof(out->path), "%s", c->path);
  out->path_len = c->path_len;
  for (int k = 0; k < 64; k++) out->node_rep[k] = k < c->path_len ? c->node_rep[k] : 0;
  return OR_OK;
}

/* ------------------------------------------------------------------ */
/* Block decompression  compress.go:34-123                             */
/* ------------------------------------------------------------------ */
/* golang/snappy decode.go Decode (block format) */
static int snappy_decode(const uint8_t *src, int64_t n, uint8_t **out, int64_t *outlen) {
  /* decodedLen: binary.Uvarint */
  uint64_t v = 0;
  int64_t s = 0;
  unsigned sh = 0;
  for (;;) {
    if (s >= n || s >= 10) return OR_ERR_DECOMPRESS;
    uint8_t b = src[s++];
    if (b < 0x80) {
      if (s == 10 && b > 1) return OR_ERR_DECOMPRESS;
      v |= (uint64_t)b << sh;
      break;
    }
    v |= (uint64_t)(b & 0x7f) << sh;
    sh += 7;
  }
  if (v > 0xffffffffULL) return OR_ERR_DECOMPRESS;
  int64_t dlen = (int64_t)v;
  uint8_t *dst = (uint8_t *)malloc((size_t)(dlen ? dlen : 1));
  if (!dst) return OR_ERR_NOMEM;
  int64_t d = 0;
  while (s < n) {
    uint8_t tag = src[s];
    int64_t length, offset;
    switch (tag & 3) {
      case 0: {
        uint32_t x = tag >> 2;
        if (x < 60) { s += 1; }
        else if (x == 60) { s += 2; if (s > n) goto corrupt; x = src[s - 1]; }
        else if (x == 61) { s += 3; if (s > n) goto corrupt; x = src[s - 2] | ((uint32_t)src[s - 1] << 8); }
        else if (x == 62) { s += 4; if (s > n) goto corrupt; x = src[s - 3] | ((uint32_t)src[s - 2] << 8) | ((uint32_t)src[s - 1] << 16); }
        else { s += 5; if (s > n) goto corrupt; x = src[s - 4] | ((uint32_t)src[s - 3] << 8) | ((uint32_t)src[s - 2] << 16) | ((uint32_t)src[s - 1] << 24); }
        length = (int64_t)x + 1;
        if (length <= 0) goto corrupt;
        if (length > dlen - d || length > n - s) goto corrupt;
        memcpy(dst + d, src + s, (size_t)length);
        d += length;
        s += length;
        continue;
      }
      case 1:
        s += 2;
        if (s > n) goto corrupt;
        length = 4 + ((src[s - 2] >> 2) & 7);
        offset = ((int64_t)(src[s - 2] & 0xe0) << 3) | src[s - 1];
        break;
      case 2:
        s += 3;
        if (s > n) goto corrupt;
        length = 1 + (src[s - 3] >> 2);
        offset = src[s - 2] | ((int64_t)src[s - 1] << 8);
        break;
      default:
        s += 5;
        if (s > n) goto corrupt;
        length = 1 + (src[s - 5] >> 2);
        offset = src[s - 4] | ((int64_t)src[s - 3] << 8) | ((int64_t)src[s - 2] << 16) | ((int64_t)src[s - 1] << 24);
        break;
    }
    if (offset <= 0 || d < offset || length > dlen - d) goto corrupt;
    for (int64_t k = 0; k < length; k++) dst[d + k] = dst[d - offset + k];
    d += length;
  }
  if (d != dlen) goto corrupt;
  *out = dst;
  *outlen = dlen;
  return OR_OK;
corrupt:
  free(dst);
  return OR_ERR_DECOMPRESS;
}

/* compress/gzip Reader (multistream) via zlib */
static int gzip_decode(const uint8_t *src, int64_t n, uint8_t **out, int64_t *outlen) {
  int64_t cap = n * 4 + 1024, len = 0;
  uint8_t *dst = (uint8_t *)malloc((size_t)cap);
  if (!dst) return OR_ERR_NOMEM;
  int64_t pos = 0;
  int members = 0;
  while (pos < n || members == 0) {
    z_stream zs;
    memset(&zs, 0, sizeof(zs));
    if (inflateInit2(&zs, 16 + MAX_WBITS) != Z_OK) { free(dst); return OR_ERR_DECOMPRESS; }
    zs.next_in = (Bytef *)(src + pos);
    zs.avail_in = (uInt)(n - pos);
    int rc;
    do {
      if (len == cap) {
        cap *= 2;
        uint8_t *nd = (uint8_t *)realloc(dst, (size_t)cap);
        if (!nd) { inflateEnd(&zs); free(dst); return OR_ERR_NOMEM; }
        dst = nd;
      }
      zs.next_out = dst + len;
      zs.avail_out = (uInt)(cap - len);
      rc = inflate(&zs, Z_NO_FLUSH);
      len = cap - zs.avail_out;
      if (rc != Z_OK && rc != Z_STREAM_END && !(rc == Z_BUF_ERROR && zs.avail_out == 0)) {
        inflateEnd(&zs); free(dst); return OR_ERR_DECOMPRESS;
      }
    } while (rc != Z_STREAM_END);
    pos = n - zs.avail_in;
    inflateEnd(&zs);
    members++;
  }
  *out = dst;
  *outlen = len;
  return OR_OK;
}

/* newBlockReader compress.go:102-123 — returns decompressed bytes (owned if *owned). */
static int new_block_reader(const uint8_t *buf, int64_t buflen, int32_t codec, int32_t csize, int32_t usize,
                            const uint8_t **res, int64_t *reslen, uint8_t **owned) {
  *owned = NULL;
  if (csize < 0 || usize < 0) return OR_ERR_INVALID;
  if (buflen != csize) return OR_ERR_INVALID;
  int e;
  if (codec == 0) { *res = buf; *reslen = buflen; }
  else if (codec == 1) {
    e = snappy_decode(buf, buflen, owned, reslen);
    if (e) return e;
    *res = *owned;
  } else if (codec == 2) {
    e = gzip_decode(buf, buflen, owned, reslen);
    if (e) return e;
    *res = *owned;
  } else return OR_ERR_UNSUPPORTED;
  if (*reslen != usize) { free(*owned); *owned = NULL; return OR_ERR_DECOMPRESS; }
  return OR_OK;
}

/* ------------------------------------------------------------------ */
/* Output accumulation (ColumnStore.readNextPage data_store.go:236-260) */
/* ------------------------------------------------------------------ */
typedef struct {
  int32_t *def, *rep;
  int64_t nslots, cap_slots;
  uint8_t *vals;
  int64_t vbytes, cap_vbytes;
  int64_t *offs;
  int64_t nvals, cap_vals;
} acc_t;

static int acc_slots(acc_t *a, int64_t add) {
  if (a->nslots + add <= a->cap_slots) return OR_OK;
  int64_t c = a->cap_slots ? a->cap_slots : 1024;
  while (c < a->nslots + add) c *= 2;
  int32_t *d = (int32_t *)realloc(a->def, sizeof(int32_t) * (size_t)c);
  if (!d) return OR_ERR_NOMEM;
  a->def = d;
  int32_t *r = (int32_t *)realloc(a->rep, sizeof(int32_t) * (size_t)c);
  if (!r) return OR_ERR_NOMEM;
  a->rep = r;
  a->cap_slots = c;
  return OR_OK;
}
static int acc_bytes(acc_t *a, const uint8_t *p, int64_t n) {
  if (a->vbytes + n > a->cap_vbytes) {
    int64_t c = a->cap_vbytes ? a->cap_vbytes : 4096;
    while (c < a->vbytes + n) c *= 2;
    uint8_t *v = (uint8_t *)realloc(a->vals, (size_t)c);
    if (!v) return OR_ERR_NOMEM;
    a->vals = v;
    a->cap_vbytes = c;
  }
  if (n) memcpy(a->vals + a->vbytes, p, (size_t)n);
  a->vbytes += n;
  return OR_OK;
}
static int acc_value(acc_t *a, const uint8_t *p, int64_t n, int track_offsets) {
  if (track_offsets) {
    if (a->nvals + 2 > a->cap_vals) {
      int64_t c = a->cap_vals ? a->cap_vals * 2 : 1024;
      int64_t *o = (int64_t *)realloc(a->offs, sizeof(int64_t) * (size_t)c);
      if (!o) return OR_ERR_NOMEM;
      a->offs = o;
      a->cap_vals = c;
    }
    if (a->nvals == 0) a->offs[0] = 0;
  }
  int e = acc_bytes(a, p, n);
  if (e) return e;
  a->nvals++;
  if (track_offsets) a->offs[a->nvals] = a->vbytes;
  return OR_OK;
}

/* ------------------------------------------------------------------ */
/* Values decoders (getValuesDecoder chunk_reader.go:106-159)          */
/* ------------------------------------------------------------------ */
enum { ENC_PLAIN = 0, ENC_PLAIN_DICT = 2, ENC_RLE = 3, ENC_BIT_PACKED = 4, ENC_DELTA_BP = 5,
       ENC_DELTA_LBA = 6, ENC_DELTA_BA = 7, ENC_RLE_DICT = 8 };
enum { T_BOOLEAN = 0, T_INT32 = 1, T_INT64 = 2, T_INT96 = 3, T_FLOAT = 4, T_DOUBLE = 5, T_BYTE_ARRAY = 6, T_FLBA = 7 };

typedef enum { VD_PLAIN_FIXED, VD_PLAIN_BOOL, VD_RLE_BOOL, VD_PLAIN_BA, VD_DELTA32, VD_DELTA64,
               VD_DELTA_LBA, VD_DELTA_BA, VD_DICT, VD_INT96 } vd_kind;

typedef struct {
  const uint8_t *p; /* dictionary payload (values concatenated) */
  int64_t *offs;    /* n+1 offsets */
  int64_t n;
} dict_t;

/* getValuesDecoder: returns the decoder kind or OR_ERR_UNSUPPORTED */
static int pick_decoder(int32_t enc, const leaf_col *c, vd_kind *k) {
  if (enc == ENC_PLAIN_DICT) enc = ENC_RLE_DICT; /* :108-110 */
  switch (c->physical_type) {
    case T_BOOLEAN:
      if (enc == ENC_PLAIN) { *k = VD_PLAIN_BOOL; return OR_OK; }
      if (enc == ENC_RLE) { *k = VD_RLE_BOOL; return OR_OK; }
      return OR_ERR_UNSUPPORTED;
    case T_BYTE_ARRAY:
      if (enc == ENC_PLAIN) { *k = VD_PLAIN_BA; return OR_OK; }
      if (enc == ENC_DELTA_LBA) { *k = VD_DELTA_LBA; return OR_OK; }
      if (enc == ENC_DELTA_BA) { *k = VD_DELTA_BA; return OR_OK; }
      if (enc == ENC_RLE_DICT) { *k = VD_DICT; return OR_OK; }
      return OR_ERR_UNSUPPORTED;
    case T_FLBA:
      if (enc == ENC_PLAIN) { *k = VD_PLAIN_BA; return OR_OK; }
      if (enc == ENC_DELTA_BA) { *k = VD_DELTA_BA; return OR_OK; }
      if (enc == ENC_RLE_DICT) { *k = VD_DICT; return OR_OK; }
      return OR_ERR_UNSUPPORTED;
    case T_FLOAT: case T_DOUBLE:
      if (enc == ENC_PLAIN) { *k = VD_PLAIN_FIXED; return OR_OK; }
      if (enc == ENC_RLE_DICT) { *k = VD_DICT; return OR_OK; }
      return OR_ERR_UNSUPPORTED;
    case T_INT96:
      if (enc == ENC_PLAIN) { *k = VD_INT96; return OR_OK; }
      if (enc == ENC_RLE_DICT) { *k = VD_DICT; return OR_OK; }
      return OR_ERR_UNSUPPORTED;
    case T_INT32: case T_INT64:
      if (enc == ENC_PLAIN) { *k = VD_PLAIN_FIXED; return OR_OK; }
      if (enc == ENC_DELTA_BP) { *k = c->physical_type == T_INT32 ? VD_DELTA32 : VD_DELTA64; return OR_OK; }
      if (enc == ENC_RLE_DICT) { *k = VD_DICT; return OR_OK; }
      return OR_ERR_UNSUPPORTED;
  }
  return OR_ERR_UNSUPPORTED;
}

static int fixed_width(int32_t t) {
  switch (t) {
    case T_INT32: case T_FLOAT: return 4;
    case T_INT64: case T_DOUBLE: return 8;
    case T_INT96: return 12;
    case T_BOOLEAN: return 1;
  }
  return 0;
}

/* byteArrayPlainDecoder.next type_bytearray.go:24-45 — returns the value slice in place */
static int ba_plain_next(breader *r, int32_t length, const uint8_t **p, int64_t *n) {
  int32_t l = length;
  int e;
  if (l == 0) {
    uint8_t b[4];
    if ((e = br_readfull(r, b, 4))) return e; /* binary.Read */
    l = (int32_t)((uint32_t)b[0] | ((uint32_t)b[1] << 8) | ((uint32_t)b[2] << 16) | ((uint32_t)b[3] << 24));
    if (l < 0) return OR_ERR_INVALID;
  } else if (l < 0) return OR_ERR_INVALID;
  int64_t start = r->i;
  if (l > 0) {
    int64_t avail = br_rem(r);
    if (avail == 0) return OR_ERR_EOF;
    if (avail < l) { r->i += avail; return OR_ERR_UNEXPECTED_EOF; }
  }
  r->i += l;
  *p = r->s + start;
  *n = l;
  return OR_OK;
}

typedef struct {
  vd_kind kind;
  const leaf_col *col;
  breader r;
  hybrid h;       /* dict keys / boolean RLE */
  delta d;        /* delta */
  int has_delta;
  const dict_t *dict;
  /* DELTA_LENGTH / DELTA_BYTE_ARRAY state */
  int32_t *lens, *prefix;
  int64_t nlens, nprefix, pos;
  uint8_t *prev;
  int64_t prevlen, prevcap;
} vdec;

static void vdec_free(vdec *v) {
  if (v->has_delta) dl_free(&v->d);
  free(v->lens);
  free(v->prefix);
  free(v->prev);
}

/* decodeInt32 helpers.go:121-131 over a fresh deltaBitPackDecoder32 */
static int decode_lengths(breader *r, int32_t **out, int64_t *n) {
  delta d;
  int e = dl_init(&d, r, 0);
  if (e) { dl_free(&d); return e; }
  int64_t cnt = d.values_count;
  int32_t *a = (int32_t *)malloc(sizeof(int32_t) * (size_t)(cnt ? cnt : 1));
  if (!a) { dl_free(&d); return OR_ERR_NOMEM; }
  for (int64_t i = 0; i < cnt; i++) {
    int64_t v;
    e = dl_next(&d, &v);
    if (e) { free(a); dl_free(&d); return e; }
    a[i] = (int32_t)v;
  }
  dl_free(&d);
  *out = a;
  *n = cnt;
  return OR_OK;
}

/* valuesDecoder.init for each kind */
static int vdec_init(vdec *v, const uint8_t *s, int64_t n) {
  br_init(&v->r, s, n);
  int e;
  switch (v->kind) {
    case VD_DICT: { /* dictDecoder.init type_dict.go:22-38 */
      uint8_t b;
      if ((e = br_readfull(&v->r, &b, 1))) return e;
      if (b > 32) return OR_ERR_INVALID;
      hyb_new(&v->h, b);
      /* keys.init(r): the keys read straight from the page reader */
      v->h.r = v->r;
      v->h.has_r = 1;
      return OR_OK;
    }
    case VD_RLE_BOOL: { /* booleanRLEDecoder.init type_boolean.go:104-107 */
      hyb_new(&v->h, 1);
      uint8_t b[4];
      if ((e = br_readfull(&v->r, b, 4))) return e;
      uint32_t size = (uint32_t)b[0] | ((uint32_t)b[1] << 8) | ((uint32_t)b[2] << 16) | ((uint32_t)b[3] << 24);
      int64_t avail = br_rem(&v->r);
      int64_t take = (int64_t)size < avail ? (int64_t)size : avail;
      hyb_init(&v->h, v->r.s + v->r.i, take);
      return OR_OK;
    }
    case VD_DELTA32: case VD_DELTA64:
      v->has_delta = 1;
      return dl_init(&v->d, &v->r, v->kind == VD_DELTA64);
    case VD_DELTA_LBA: /* byteArrayDeltaLengthDecoder.init type_bytearray.go:104-115 */
      v->pos = 0;
      return decode_lengths(&v->r, &v->lens, &v->nlens);
    case VD_DELTA_BA: /* byteArrayDeltaDecoder.init :195-214 */
      if ((e = decode_lengths(&v->r, &v->prefix, &v->nprefix))) return e;
      v->pos = 0;
      if ((e = decode_lengths(&v->r, &v->lens, &v->nlens))) return e;
      if (v->nprefix != v->nlens) return OR_ERR_INVALID;
      v->prevlen = 0;
      return OR_OK;
    default:
      return OR_OK;
  }
}

/* decodeValues for nn values, appending to acc. Returns err class. */
static int vdec_decode(vdec *v, int64_t nn, acc_t *a) {
  const leaf_col *c = v->col;
  int e;
  int is_ba = c->physical_type == T_BYTE_ARRAY || c->physical_type == T_FLBA;
  switch (v->kind) {
    case VD_PLAIN_FIXED: { /* type_int32.go:21-31 etc: binary.Read per value */
      int w = fixed_width(c->physical_type);
      uint8_t b[8];
      for (int64_t i = 0; i < nn; i++) {
        if ((e = br_readfull(&v->r, b, w))) return e;
        if ((e = acc_value(a, b, w, 0))) return e;
      }
      return OR_OK;
    }
    case VD_INT96: { /* int96PlainDecoder.decodeValues type_int96.go:21-42 (Q6) */
      for (int64_t i = 0; i < nn; i++) {
        uint8_t b[12];
        int64_t got;
        int er = br_read(&v->r, b, 12, &got);
        if (got == 12) { if ((e = acc_value(a, b, 12, 0))) return e; }
        if (er && (got == 0 || got == 12)) return er;
        if (er) return OR_ERR_INVALID;
      }
      return OR_OK;
    }
    case VD_PLAIN_BOOL: { /* booleanPlainDecoder.decodeValues type_boolean.go:46-69 */
      for (int64_t i = 0; i < nn; i += 8) {
        uint8_t b;
        if ((e = br_readfull(&v->r, &b, 1))) return e;
        for (int j = 0; j < 8 && i + j < nn; j++) {
          uint8_t bit = (b >> j) & 1;
          if ((e = acc_value(a, &bit, 1, 0))) return e;
        }
      }
      return OR_OK;
    }
    case VD_RLE_BOOL: { /* booleanRLEDecoder.decodeValues :109-120 */
      for (int64_t i = 0; i < nn; i++) {
        int32_t x;
        if ((e = hyb_next(&v->h, &x))) return e;
        uint8_t bit = x == 1;
        if ((e = acc_value(a, &bit, 1, 0))) return e;
      }
      return OR_OK;
    }
    case VD_PLAIN_BA: {
      for (int64_t i = 0; i < nn; i++) {
        const uint8_t *p; int64_t n;
        if ((e = ba_plain_next(&v->r, c->physical_type == T_FLBA ? c->type_length : 0, &p, &n))) return e;
        if ((e = acc_value(a, p, n, 1))) return e;
      }
      return OR_OK;
    }
    case VD_DELTA32: case VD_DELTA64: { /* type_int32.go:59-69 / type_int64.go:59-69 */
      for (int64_t i = 0; i < nn; i++) {
        int64_t x;
        if ((e = dl_next(&v->d, &x))) return e;
        if (v->kind == VD_DELTA32) {
          int32_t y = (int32_t)x;
          if ((e = acc_value(a, (uint8_t *)&y, 4, 0))) return e;
        } else {
          if ((e = acc_value(a, (uint8_t *)&x, 8, 0))) return e;
        }
      }
      return OR_OK;
    }
    case VD_DELTA_LBA: { /* byteArrayDeltaLengthDecoder.next :117-140 */
      for (int64_t i = 0; i < nn; i++) {
        if (v->pos >= v->nlens) return OR_ERR_EOF;
        int64_t size = v->lens[v->pos];
        if (size < 0) return OR_ERR_INVALID; /* make([]byte, negative) panics in Go */
        int64_t avail = br_rem(&v->r);
        if (size > 0 && avail == 0) return OR_ERR_EOF;
        if (size > avail) return OR_ERR_UNEXPECTED_EOF;
        const uint8_t *p = v->r.s + v->r.i;
        v->r.i += size;
        v->pos++;
        if ((e = acc_value(a, p, size, 1))) return e;
      }
      return OR_OK;
    }
    case VD_DELTA_BA: { /* byteArrayDeltaDecoder.decodeValues :216-240 */
      for (int64_t i = 0; i < nn; i++) {
        if (v->pos >= v->nlens) return OR_ERR_EOF;
        int64_t size = v->lens[v->pos];
        if (size < 0) return OR_ERR_INVALID;
        int64_t avail = br_rem(&v->r);
        if (size > 0 && avail == 0) return OR_ERR_EOF;
        if (size > avail) return OR_ERR_UNEXPECTED_EOF;
        const uint8_t *suffix = v->r.s + v->r.i;
        v->r.i += size;
        v->pos++;
        int64_t pl = v->prefix[v->pos - 1];
        /* make([]byte, 0, prefixLen+len(suffix)) panics on a negative capacity (reported as
           invalid); a negative prefix with a long enough suffix appends nothing of the
           previous value (:224-235) */
        if (pl + size < 0) return OR_ERR_INVALID;
        if (v->prevlen < pl) return OR_ERR_INVALID;
        if (pl < 0) pl = 0;
        int64_t nl = pl + size;
        uint8_t *nv = (uint8_t *)malloc((size_t)(nl ? nl : 1));
        if (!nv) return OR_ERR_NOMEM;
        if (pl) memcpy(nv, v->prev, (size_t)pl);
        if (size) memcpy(nv + pl, suffix, (size_t)size);
        free(v->prev);
        v->prev = nv;
        v->prevlen = nl;
        if ((e = acc_value(a, nv, nl, 1))) return e;
      }
      return OR_OK;
    }
    case VD_DICT: { /* dictDecoder.decodeValues type_dict.go:40-60 */
      const dict_t *d = v->dict;
      int64_t size = d ? d->n : 0;
      for (int64_t i = 0; i < nn; i++) {
        int32_t key;
        if ((e = hyb_next(&v->h, &key))) return e;
        if (key < 0 || key >= size) return OR_ERR_DICT_INDEX;
        const uint8_t *p = d->p + d->offs[key];
        int64_t n = d->offs[key + 1] - d->offs[key];
        if ((e = acc_value(a, p, n, is_ba))) return e;
      }
      return OR_OK;
    }
  }
  return OR_ERR_UNSUPPORTED;
}

/* ------------------------------------------------------------------ */
/* Chunk reader  chunk_reader.go:182-404, page_v1.go, page_v2.go       */
/* ------------------------------------------------------------------ */
typedef struct {
  int v2;
  int32_t num_values;
  /* level streams (already sliced) */
  const uint8_t *rep_s; int64_t rep_n; int rep_has;
  const uint8_t *def_s; int64_t def_n; int def_has;
  vdec vd;
  uint8_t *owned;  /* decompressed block */
  uint8_t *owned2;
} page_t;

static uint32_t crc32_ieee(const uint8_t *p, int64_t n) { return (uint32_t)crc32(0L, p, (uInt)n); }

/* bits.Len16 */
static int bits_len16(int v) { int n = 0; while (v) { n++; v >>= 1; } return n; }

/* readPageBlock chunk_reader.go:161-180 over the file offsetReader */
static int read_page_block(const or_file *f, int64_t *off, int64_t *count, int32_t csize, int32_t usize, int validate,
                           int has_crc, int32_t crc, const uint8_t **blk, int64_t *blklen) {
  if (csize < 0 || usize < 0) return OR_ERR_INVALID;
  int64_t avail = *off >= f->len ? 0 : f->len - *off;
  int64_t take = (int64_t)csize < avail ? (int64_t)csize : avail;
  *blk = f->buf + (*off < f->len ? *off : f->len);
  *blklen = take;
  *off += take;
  *count += take;
  if (validate && has_crc) {
    if (crc32_ieee(*blk, take) != (uint32_t)crc) return OR_ERR_CRC;
  }
  return OR_OK;
}

/* readValues(size) page_v1.go:33-63 / page_v2.go:31-60 */
static int page_read_values(page_t *p, const leaf_col *c, acc_t *a) {
  int64_t size = p->num_values;
  if (size == 0) return OR_OK;
  int e;
  if ((e = acc_slots(a, size))) return e;
  int rbw = bits_len16(c->max_rep), dbw = bits_len16(c->max_def);
  hybrid hr, hd;
  hyb_new(&hr, rbw);
  hyb_new(&hd, dbw);
  if (p->rep_has) hyb_init(&hr, p->rep_s, p->rep_n);
  if (p->def_has) hyb_init(&hd, p->def_s, p->def_n);
  /* rep levels: decodePackedArray helpers.go:133-149 (constDecoder(0) when maxR == 0) */
  for (int64_t i = 0; i < size; i++) {
    int32_t x = 0;
    if (c->max_rep > 0 && (e = hyb_next(&hr, &x))) return e;
    a->rep[a->nslots + i] = x;
  }
  int64_t nn = 0;
  for (int64_t i = 0; i < size; i++) {
    int32_t x = 0;
    if (c->max_def > 0 && (e = hyb_next(&hd, &x))) return e;
    a->def[a->nslots + i] = x;
    if (x == c->max_def) nn++;
  }
  a->nslots += size;
  if (nn != 0) {
    if ((e = vdec_decode(&p->vd, nn, a))) return e;
  }
  return OR_OK;
}

static void page_free(page_t *p) {
  vdec_free(&p->vd);
  free(p->owned);
  free(p->owned2);
}

/* readChunk :299-362 + readPages :182-263 + readValues for every page */
int or_read_chunk(const or_file *f, int rg, int col, int validate_crc, or_chunk_result *out) {
  memset(out, 0, sizeof(*out));
  out->err_page = -1;
  if (rg < 0 || rg >= f->nrgs) { out->err_code = OR_ERR_ARG; return OR_ERR_ARG; }
  const row_group *g = &f->rgs[rg];
  if (col < 0 || col >= f->nleaves) { out->err_code = OR_ERR_ARG; return OR_ERR_ARG; }
  const leaf_col *c = &f->leaves[col];
  out->value_width = (c->physical_type == T_BYTE_ARRAY || c->physical_type == T_FLBA) ? 0 : fixed_width(c->physical_type);
  int e = OR_OK;
  page_t **pages = NULL; /* individually allocated: decoders keep pointers into their page */
  int npages = 0, cap = 0;
  dict_t dict = {0};
  int64_t *dict_offs = NULL;
  acc_t dacc = {0};
  int has_dict = 0;
  acc_t a = {0};

#define FAIL(code, page, msg) do { e = (code); out->err_page = (page); snprintf(out->err_msg, sizeof(out->err_msg), "%s", msg); goto done; } while (0)
  if (g->ncols <= col) FAIL(OR_ERR_INVALID, -1, "column index out of bounds");
  const col_chunk *cc = &g->cols[col];
  if (cc->has_file_path) FAIL(OR_ERR_UNSUPPORTED, -1, "nyi: data is in another file");
  if (!cc->has_meta) FAIL(OR_ERR_INVALID, -1, "missing meta data for Column");
  if (cc->type != c->physical_type) FAIL(OR_ERR_INVALID, -1, "wrong type in Column chunk metadata");
  int64_t off = cc->data_page_offset;
  if (cc->has_dict_offset) off = cc->dict_offset;
  if (off < 0) FAIL(OR_ERR_INVALID, -1, "seek: negative position");
  int64_t count = 0;
  for (;;) {
    if (cc->total_compressed - count <= 0) break;
    page_header_t ph;
    breader hr;
    br_init(&hr, f->buf, f->len);
    hr.i = off;
    e = rd_page_header(&hr, &ph);
    int64_t consumed = (hr.i < f->len ? hr.i : f->len) - off;
    if (consumed < 0) consumed = 0;
    off += consumed;
    count += consumed;
    if (e) FAIL(e, -1, "thrift: page header");
    if (ph.type == 2) { /* DICTIONARY_PAGE page_dict.go:35-72 */
      if (has_dict) FAIL(OR_ERR_INVALID, -1, "there should be only one dictionary");
      vd_kind dk;
      if (c->physical_type == T_BOOLEAN) FAIL(OR_ERR_UNSUPPORTED, -1, "type not supported for dict value encoder");
      if (c->physical_type == T_FLBA && c->type_length == 0) FAIL(OR_ERR_INVALID, -1, "nil type len");
      dk = (c->physical_type == T_BYTE_ARRAY || c->physical_type == T_FLBA) ? VD_PLAIN_BA
           : (c->physical_type == T_INT96 ? VD_INT96 : VD_PLAIN_FIXED);
      if (!ph.has_dict) FAIL(OR_ERR_INVALID, -1, "null DictionaryPageHeader");
      if (ph.dict.num_values < 0) FAIL(OR_ERR_INVALID, -1, "negative NumValues in DICTIONARY_PAGE");
      if (ph.dict.encoding != ENC_PLAIN && ph.dict.encoding != ENC_PLAIN_DICT)
        FAIL(OR_ERR_UNSUPPORTED, -1, "only Encoding_PLAIN and Encoding_PLAIN_DICTIONARY is supported");
      const uint8_t *blk; int64_t blen;
      if ((e = read_page_block(f, &off, &count, ph.csize, ph.usize, validate_crc, ph.has_crc, ph.crc, &blk, &blen)))
        FAIL(e, -1, "dictionary page block");
      const uint8_t *res; int64_t rlen; uint8_t *owned;
      if ((e = new_block_reader(blk, blen, cc->codec, ph.csize, ph.usize, &res, &rlen, &owned)))
        FAIL(e, -1, "dictionary page decompress");
      vdec vd;
      memset(&vd, 0, sizeof(vd));
      vd.kind = dk;
      vd.col = c;
      vdec_init(&vd, res, rlen);
      acc_t tmp = {0};
      int is_ba = dk == VD_PLAIN_BA;
      /* decode NumValues entries; each stored with offsets so the dict can gather */
      leaf_col fake = *c;
      vd.col = &fake;
      if (!is_ba) {
        /* fixed width: record offsets manually */
        e = vdec_decode(&vd, ph.dict.num_values, &tmp);
      } else {
        e = vdec_decode(&vd, ph.dict.num_values, &tmp);
      }
      vdec_free(&vd);
      if (!e && dk == VD_INT96 && tmp.nvals != ph.dict.num_values) {
        /* Q6: truncated INT96 entries stay nil in the dictionary; represent as error-free short dict */
      }
      if (e) { free(owned); free(tmp.vals); free(tmp.offs); free(tmp.def); free(tmp.rep); FAIL(e, -1, "dictionary decode"); }
      dacc = tmp;
      dict.n = tmp.nvals;
      dict.p = dacc.vals;
      if (is_ba) {
        if (tmp.nvals == 0) {
          dict_offs = (int64_t *)calloc(1, sizeof(int64_t));
          free(dacc.offs);
          dacc.offs = NULL;
        } else {
          dict_offs = dacc.offs;
          dacc.offs = NULL;
        }
      } else {
        int w = fixed_width(c->physical_type);
        dict_offs = (int64_t *)malloc(sizeof(int64_t) * (size_t)(tmp.nvals + 1));
        for (int64_t i = 0; i <= tmp.nvals; i++) dict_offs[i] = i * w;
      }
      dict.offs = dict_offs;
      free(owned);
      has_dict = 1;
      if (cc->has_dict_offset && cc->dict_offset != off) {
        int64_t np = cc->data_page_offset;
        if (np < 0) FAIL(OR_ERR_INVALID, -1, "seek: negative position");
        count += np - off;
        off = np;
      }
      continue;
    }
    if (ph.type != 0 && ph.type != 3) FAIL(OR_ERR_UNSUPPORTED, -1, "DATA_PAGE or DATA_PAGE_V2 type supported");
    if (npages == cap) {
      cap = cap ? cap * 2 : 16;
      page_t **np = (page_t **)realloc(pages, sizeof(page_t *) * (size_t)cap);
      if (!np) FAIL(OR_ERR_NOMEM, -1, "nomem");
      pages = np;
    }
    page_t *p = (page_t *)calloc(1, sizeof(page_t));
    if (!p) FAIL(OR_ERR_NOMEM, -1, "nomem");
    pages[npages] = p;
    p->vd.col = c;
    p->vd.dict = &dict;
    npages++;
    int pi = npages - 1;
    if (ph.type == 0) {
      /* dataPageReaderV1.init page_v1.go:65-85: level decoders */
      if (!ph.has_dph) FAIL(OR_ERR_INVALID, pi, "page header is missing data page header");
      if (c->max_rep > 0 && ph.dph.rep_enc != ENC_RLE) FAIL(OR_ERR_UNSUPPORTED, pi, "not supported for repetition level");
      if (c->max_def > 0 && ph.dph.def_enc != ENC_RLE) FAIL(OR_ERR_UNSUPPORTED, pi, "not supported for definition level");
      /* read :87-122 */
      if ((p->num_values = ph.dph.num_values) < 0) FAIL(OR_ERR_INVALID, pi, "negative NumValues in DATA_PAGE");
      const uint8_t *blk; int64_t blen;
      if ((e = read_page_block(f, &off, &count, ph.csize, ph.usize, validate_crc, ph.has_crc, ph.crc, &blk, &blen)))
        FAIL(e, pi, "page block");
      const uint8_t *res; int64_t rlen;
      if ((e = new_block_reader(blk, blen, cc->codec, ph.csize, ph.usize, &res, &rlen, &p->owned)))
        FAIL(e, pi, "page decompress");
      vd_kind k;
      if ((e = pick_decoder(ph.dph.encoding, c, &k))) FAIL(e, pi, "unsupported encoding");
      p->vd.kind = k;
      breader pr;
      br_init(&pr, res, rlen);
      /* rDecoder.initSize / dDecoder.initSize: u32 length + LimitReader + ReadAll */
      if (c->max_rep > 0) {
        uint8_t b[4];
        if ((e = br_readfull(&pr, b, 4))) FAIL(e, pi, "rep level size");
        uint32_t sz = (uint32_t)b[0] | ((uint32_t)b[1] << 8) | ((uint32_t)b[2] << 16) | ((uint32_t)b[3] << 24);
        int64_t take = (int64_t)sz < br_rem(&pr) ? (int64_t)sz : br_rem(&pr);
        p->rep_s = pr.s + pr.i; p->rep_n = take; p->rep_has = 1;
        pr.i += take;
      }
      if (c->max_def > 0) {
        uint8_t b[4];
        if ((e = br_readfull(&pr, b, 4))) FAIL(e, pi, "def level size");
        uint32_t sz = (uint32_t)b[0] | ((uint32_t)b[1] << 8) | ((uint32_t)b[2] << 16) | ((uint32_t)b[3] << 24);
        int64_t take = (int64_t)sz < br_rem(&pr) ? (int64_t)sz : br_rem(&pr);
        p->def_s = pr.s + pr.i; p->def_n = take; p->def_has = 1;
        pr.i += take;
      }
      if ((e = vdec_init(&p->vd, pr.s + pr.i, pr.n - pr.i))) FAIL(e, pi, "values decoder init");
    } else {
      /* dataPageReaderV2.read page_v2.go:79-131 */
      p->v2 = 1;
      if (!ph.has_dph2) FAIL(OR_ERR_INVALID, pi, "null DataPageHeaderV2");
      if ((p->num_values = ph.dph2.num_values) < 0) FAIL(OR_ERR_INVALID, pi, "negative NumValues in DATA_PAGE_V2");
      if (ph.dph2.rep_len < 0) FAIL(OR_ERR_INVALID, pi, "invalid RepetitionLevelsByteLength");
      if (ph.dph2.def_len < 0) FAIL(OR_ERR_INVALID, pi, "invalid DefinitionLevelsByteLength");
      vd_kind k;
      if ((e = pick_decoder(ph.dph2.encoding, c, &k))) FAIL(e, pi, "unsupported encoding");
      p->vd.kind = k;
      const uint8_t *blk; int64_t blen;
      if ((e = read_page_block(f, &off, &count, ph.csize, ph.usize, validate_crc, ph.has_crc, ph.crc, &blk, &blen)))
        FAIL(e, pi, "page block");
      int64_t rl = ph.dph2.rep_len, dl = ph.dph2.def_len;
      int64_t levels = rl + dl;
      /* Go would panic on these slice bounds (runtime.Error); reported as invalid here */
      if (rl > blen || levels > blen) FAIL(OR_ERR_INVALID, pi, "slice bounds out of range");
      if (rl > 0 && c->max_rep > 0) { p->rep_s = blk; p->rep_n = rl; p->rep_has = 1; }
      if (dl > 0 && c->max_def > 0) { p->def_s = blk + rl; p->def_n = dl; p->def_has = 1; }
      const uint8_t *res; int64_t rlen;
      int64_t cs2 = (int64_t)ph.csize - levels, us2 = (int64_t)ph.usize - levels;
      if (cs2 < 0 || us2 < 0) FAIL(OR_ERR_INVALID, pi, "invalid page data size");
      if ((e = new_block_reader(blk + levels, blen - levels, cc->codec, (int32_t)cs2, (int32_t)us2, &res, &rlen, &p->owned)))
        FAIL(e, pi, "page decompress");
      if ((e = vdec_init(&p->vd, res, rlen))) FAIL(e, pi, "values decoder init");
    }
  }
  /* readPageData + ColumnStore.get -> readNextPage, every page in order */
  for (int i = 0; i < npages; i++) {
    if ((e = page_read_values(pages[i], c, &a))) {
      out->err_page = i;
      snprintf(out->err_msg, sizeof(out->err_msg), "read values from page failed");
      goto done;
    }
  }
done:
#undef FAIL
  for (int i = 0; i < npages; i++) { page_free(pages[i]); free(pages[i]); }
  free(pages);
  free(dict_offs);
  free(dacc.vals); free(dacc.offs); free(dacc.def); free(dacc.rep);
  out->num_pages = npages;
  out->err_code = e;
  if (e) {
    free(a.def); free(a.rep); free(a.vals); free(a.offs);
    return e;
  }
  out->num_slots = a.nslots;
  out->num_values = a.nvals;
  out->def_levels = a.def;
  out->rep_levels = a.rep;
  out->values = a.vals;
  out->values_bytes = a.vbytes;
  if (out->value_width == 0) {
    if (a.nvals == 0) { free(a.offs); a.offs = (int64_t *)calloc(1, sizeof(int64_t)); }
    out->offsets = a.offs;
  } else {
    free(a.offs);
  }
  return OR_OK;
}

void or_chunk_result_free(or_chunk_result *r) {
  free(r->def_levels);
  free(r->rep_levels);
  free(r->values);
  free(r->offsets);
  memset(r, 0, sizeof(*r));
}
