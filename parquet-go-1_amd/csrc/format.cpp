// format.cpp — Thrift compact reader, Parquet footer/schema, page headers,
// host SNAPPY/GZIP. See format.h. Error classes follow include/pqgpu.h.
#include "format.h"

#include <string.h>

#include <algorithm>
#include <array>
#include <zlib.h>

#include "../../include/pqgpu.h"
#include "pq_device.h"

namespace pq {

// ---------------------------------------------------------------------------
// Thrift compact protocol
// ---------------------------------------------------------------------------
enum { CT_STOP = 0, CT_TRUE = 1, CT_FALSE = 2, CT_BYTE = 3, CT_I16 = 4, CT_I32 = 5, CT_I64 = 6, CT_DOUBLE = 7,
       CT_BINARY = 8, CT_LIST = 9, CT_SET = 10, CT_MAP = 11, CT_STRUCT = 12 };

bool ThriftReader::byte(uint8_t *b) {
  if (err_ || i_ >= n_) { err_ = true; return false; }
  *b = p_[i_++];
  return true;
}

uint64_t ThriftReader::uvarint() {
  uint64_t x = 0;
  unsigned s = 0;
  for (;;) {
    uint8_t b;
    if (!byte(&b)) return 0;
    if (s < 64) x |= (uint64_t)(b & 0x7f) << s;
    if (!(b & 0x80)) return x;
    s += 7;
  }
}

bool ThriftReader::binary(std::string *out) {
  int32_t len = (int32_t)uvarint();
  if (err_) return false;
  if (len < 0 || (int64_t)len > n_ - i_) { err_ = true; return false; }
  if (out) out->assign((const char *)p_ + i_, (size_t)len);
  i_ += len;
  return true;
}

bool ThriftReader::list_begin(int *etype, int32_t *size) {
  uint8_t b;
  if (!byte(&b)) return false;
  int32_t sz = (b >> 4) & 0x0f;
  if (sz == 15) sz = (int32_t)uvarint();
  if (err_ || sz < 0 || (b & 0x0f) > CT_STRUCT) { err_ = true; return false; }  // getTType: unknown type
  *etype = b & 0x0f;
  *size = sz;
  return true;
}

bool ThriftReader::field(int16_t *last, int16_t *id, int *type) {
  uint8_t b;
  if (!byte(&b)) return false;
  if ((b & 0x0f) == CT_STOP) return false;
  int mod = b >> 4;
  *id = mod ? (int16_t)(*last + mod) : (int16_t)i32();
  if (err_) return false;
  *last = *id;
  *type = b & 0x0f;
  if (*type > CT_STRUCT) { err_ = true; return false; }
  return true;
}

void ThriftReader::skip(int type, int depth) {
  if (err_) return;
  if (depth > 64) { err_ = true; return; }
  uint8_t b;
  switch (type) {
    case CT_TRUE: case CT_FALSE: case CT_BYTE: byte(&b); break;
    case CT_I16: case CT_I32: case CT_I64: uvarint(); break;
    case CT_DOUBLE:
      if (n_ - i_ < 8) err_ = true; else i_ += 8;
      break;
    case CT_BINARY: binary(nullptr); break;
    case CT_LIST: case CT_SET: {
      int et; int32_t n;
      if (!list_begin(&et, &n)) return;
      for (int32_t k = 0; k < n && !err_; k++) skip(et, depth + 1);
      break;
    }
    case CT_MAP: {
      int32_t n = (int32_t)uvarint();
      if (err_) return;
      if (n < 0) { err_ = true; return; }
      if (n == 0) break;
      if (!byte(&b)) return;
      for (int32_t k = 0; k < n && !err_; k++) { skip(b >> 4, depth + 1); skip(b & 0x0f, depth + 1); }
      break;
    }
    case CT_STRUCT: {
      int16_t last = 0, id;
      int ty;
      while (field(&last, &id, &ty)) {
        if (ty != CT_TRUE && ty != CT_FALSE) skip(ty, depth + 1);
      }
      break;
    }
    default: err_ = true;
  }
}

static inline void skip_field(ThriftReader &t, int ty) {
  if (ty != CT_TRUE && ty != CT_FALSE) t.skip(ty, 1);
}

// ---------------------------------------------------------------------------
// PageHeader (parquet.thrift) — required fields checked like the generated Go code.
// ---------------------------------------------------------------------------
bool ParsePageHeader(const uint8_t *p, int64_t n, PageHeader *h, int64_t *consumed) {
  *h = PageHeader();
  ThriftReader t(p, n);
  int16_t last = 0, id;
  int ty;
  bool st = false, su = false, sc = false;
  while (t.field(&last, &id, &ty)) {
    if (id == 1 && ty == CT_I32) { h->type = t.i32(); st = true; }
    else if (id == 2 && ty == CT_I32) { h->usize = t.i32(); su = true; }
    else if (id == 3 && ty == CT_I32) { h->csize = t.i32(); sc = true; }
    else if (id == 4 && ty == CT_I32) { h->crc = t.i32(); h->has_crc = true; }
    else if (id == 5 && ty == CT_STRUCT) {
      h->has_dph = true;
      int16_t l2 = 0, i2; int t2;
      bool a = false, b = false, c = false, d = false;
      while (t.field(&l2, &i2, &t2)) {
        if (i2 == 1 && t2 == CT_I32) { h->dph.num_values = t.i32(); a = true; }
        else if (i2 == 2 && t2 == CT_I32) { h->dph.encoding = t.i32(); b = true; }
        else if (i2 == 3 && t2 == CT_I32) { h->dph.def_enc = t.i32(); c = true; }
        else if (i2 == 4 && t2 == CT_I32) { h->dph.rep_enc = t.i32(); d = true; }
        else skip_field(t, t2);
      }
      if (!t.failed() && !(a && b && c && d)) t.fail();
    } else if (id == 7 && ty == CT_STRUCT) {
      h->has_dict = true;
      int16_t l2 = 0, i2; int t2;
      bool a = false, b = false;
      while (t.field(&l2, &i2, &t2)) {
        if (i2 == 1 && t2 == CT_I32) { h->dict.num_values = t.i32(); a = true; }
        else if (i2 == 2 && t2 == CT_I32) { h->dict.encoding = t.i32(); b = true; }
        else skip_field(t, t2);
      }
      if (!t.failed() && !(a && b)) t.fail();
    } else if (id == 8 && ty == CT_STRUCT) {
      h->has_dph2 = true;
      int16_t l2 = 0, i2; int t2;
      unsigned set = 0;
      while (t.field(&l2, &i2, &t2)) {
        if (t2 == CT_I32 && i2 >= 1 && i2 <= 6) {
          int32_t v = t.i32();
          set |= 1u << i2;
          switch (i2) {
            case 1: h->dph2.num_values = v; break;
            case 2: h->dph2.num_nulls = v; break;
            case 3: h->dph2.num_rows = v; break;
            case 4: h->dph2.encoding = v; break;
            case 5: h->dph2.def_len = v; break;
            case 6: h->dph2.rep_len = v; break;
          }
        } else if (i2 == 7 && (t2 == CT_TRUE || t2 == CT_FALSE)) {
          h->dph2.is_compressed = t2 == CT_TRUE;
        } else skip_field(t, t2);
      }
      if (!t.failed() && set != 0x7e) t.fail();
    } else skip_field(t, ty);
  }
  if (!t.failed() && !(st && su && sc)) t.fail();
  *consumed = t.pos();
  return !t.failed();
}

// ---------------------------------------------------------------------------
// FileMetaData
// ---------------------------------------------------------------------------
static void read_schema_element(ThriftReader &t, SchemaElement *e) {
  int16_t last = 0, id;
  int ty;
  bool has_name = false;
  while (t.field(&last, &id, &ty)) {
    if (id == 1 && ty == CT_I32) { e->type = t.i32(); e->has_type = true; }
    else if (id == 2 && ty == CT_I32) { e->type_length = t.i32(); e->has_type_length = true; }
    else if (id == 3 && ty == CT_I32) { e->rep = t.i32(); e->has_rep = true; }
    else if (id == 4 && ty == CT_BINARY) { t.binary(&e->name); has_name = true; }
    else if (id == 5 && ty == CT_I32) { e->num_children = t.i32(); e->has_num_children = true; }
    else skip_field(t, ty);
  }
  if (!t.failed() && !has_name) t.fail();
}

static void read_column_meta(ThriftReader &t, ColumnChunkMeta *c) {
  int16_t last = 0, id;
  int ty;
  unsigned set = 0;
  while (t.field(&last, &id, &ty)) {
    if (id == 1 && ty == CT_I32) { c->type = t.i32(); set |= 1; }
    else if (id == 2 && ty == CT_LIST) { t.skip(ty, 1); set |= 2; }
    else if (id == 3 && ty == CT_LIST) { t.skip(ty, 1); set |= 4; }
    else if (id == 4 && ty == CT_I32) { c->codec = t.i32(); set |= 8; }
    else if (id == 5 && ty == CT_I64) { c->num_values = t.i64(); set |= 16; }
    else if (id == 6 && ty == CT_I64) { c->total_uncompressed = t.i64(); set |= 32; }
    else if (id == 7 && ty == CT_I64) { c->total_compressed = t.i64(); set |= 64; }
    else if (id == 9 && ty == CT_I64) { c->data_page_offset = t.i64(); set |= 128; }
    else if (id == 11 && ty == CT_I64) { c->dict_offset = t.i64(); c->has_dict_offset = true; }
    else skip_field(t, ty);
  }
  if (!t.failed() && set != 255) t.fail();
}

static void read_column_chunk(ThriftReader &t, ColumnChunkMeta *c) {
  int16_t last = 0, id;
  int ty;
  bool fo = false;
  while (t.field(&last, &id, &ty)) {
    if (id == 1 && ty == CT_BINARY) { c->has_file_path = true; t.binary(nullptr); }
    else if (id == 2 && ty == CT_I64) { t.i64(); fo = true; }
    else if (id == 3 && ty == CT_STRUCT) { c->has_meta = true; read_column_meta(t, c); }
    else skip_field(t, ty);
  }
  if (!t.failed() && !fo) t.fail();
}

template <class T, class F>
static bool read_struct_list(ThriftReader &t, std::vector<T> *v, F fn, int64_t remaining) {
  int et;
  int32_t n;
  // parquet.go's generated ReadFieldN discards ReadListBegin's element type and reads every
  // element as the field's struct type
  if (!t.list_begin(&et, &n)) return false;
  if ((int64_t)n > remaining) { t.fail(); return false; }
  v->resize((size_t)n);
  for (int32_t k = 0; k < n && !t.failed(); k++) fn(t, &(*v)[(size_t)k]);
  return !t.failed();
}

static void read_row_group(ThriftReader &t, RowGroup *g, int64_t remaining) {
  int16_t last = 0, id;
  int ty;
  unsigned set = 0;
  while (t.field(&last, &id, &ty)) {
    if (id == 1 && ty == CT_LIST) {
      read_struct_list(t, &g->cols, read_column_chunk, remaining);
      set |= 1;
    } else if (id == 2 && ty == CT_I64) { t.i64(); set |= 2; }
    else if (id == 3 && ty == CT_I64) { g->num_rows = t.i64(); set |= 4; }
    else skip_field(t, ty);
  }
  if (!t.failed() && set != 7) t.fail();
}

// schema.go:893-924 readColumnSchema
// `lists`: (definition level before, at) of every REPEATED ancestor, outermost first;
// `groups`: (definition level, REPEATED ancestors above, path position) of every OPTIONAL group ancestor
using ListLevels = std::vector<std::array<int32_t, 3>>;  // + the node's path position
using GroupLevels = std::vector<std::array<int32_t, 3>>;
static Status read_column_schema(FileMeta *f, size_t base, int32_t idx, const std::string &path, int d, int r,
                                 int32_t *next, const ListLevels &lists, const GroupLevels &groups) {
  const SchemaElement &s = f->schema[base + (size_t)idx];
  if (s.name.empty()) return Status::Err(PQ_ERR_INVALID, "name in schema is empty");
  if (!s.has_rep) return Status::Err(PQ_ERR_INVALID, "field RepetitionType is nil");
  const int d0 = d;
  if (s.rep != 0) d++;
  if (s.rep == 2) r++;
  Leaf l;
  const int32_t self = (int32_t)std::count(path.begin(), path.end(), '.') + (path.empty() ? 0 : 1);
  for (const auto &x : lists) { l.list_null_def.push_back(x[0]); l.list_def.push_back(x[1]); l.list_node.push_back(x[2]); }
  if (s.rep == 2) { l.list_null_def.push_back(d0); l.list_def.push_back(d); l.list_node.push_back(self); }
  for (const auto &g : groups) { l.group_def.push_back(g[0]); l.group_depth.push_back(g[1]); l.group_node.push_back(g[2]); }
  l.type = s.type;
  l.type_length = s.has_type_length ? s.type_length : 0;
  l.max_def = d;
  l.max_rep = r;
  l.rep = s.rep;
  l.path = path.empty() ? s.name : path + "." + s.name;
  if (s.type < 0 || s.type > 7) return Status::Err(PQ_ERR_UNSUPPORTED, "unsupported type");
  if (s.type == T_FLBA && !s.has_type_length) return Status::Err(PQ_ERR_INVALID, "type with nil type length");
  f->leaves.push_back(l);
  *next = idx + 1;
  return Status::Ok();
}

// schema.go:926-990 readGroupSchema
static Status read_group_schema(FileMeta *f, size_t base, int32_t n, int32_t idx, const std::string &path, int d,
                                int r, int32_t *next, int depth, const ListLevels &lists, const GroupLevels &groups) {
  if (depth > 1000 || n <= idx) return Status::Err(PQ_ERR_INVALID, "schema index out of bound");
  const SchemaElement &s = f->schema[base + (size_t)idx];
  if (s.has_type) return Status::Err(PQ_ERR_INVALID, "field Type is not nil");
  if (!s.has_num_children) return Status::Err(PQ_ERR_INVALID, "the field NumChildren is invalid");
  if (s.num_children <= 0) return Status::Err(PQ_ERR_INVALID, "the field NumChildren is zero");
  int32_t l = s.num_children;
  if ((int64_t)n <= (int64_t)idx + l) return Status::Err(PQ_ERR_INVALID, "not enough element in the schema list");
  const int d0 = d;
  if (s.has_rep && s.rep != 0) d++;
  if (s.has_rep && s.rep == 2) r++;
  ListLevels sub = lists;
  if (s.has_rep && s.rep == 2) sub.push_back({d0, d, depth});
  GroupLevels gsub = groups;
  if (s.has_rep && s.rep == 1) gsub.push_back({d, r, depth});
  std::string p = path.empty() ? s.name : path + "." + s.name;
  idx++;
  for (int32_t k = 0; k < l; k++) {
    if (n <= idx) return Status::Err(PQ_ERR_INVALID, "schema index is out of bounds");
    Status st = !f->schema[base + (size_t)idx].has_type ? read_group_schema(f, base, n, idx, p, d, r, &idx, depth + 1, sub, gsub)
                                                        : read_column_schema(f, base, idx, p, d, r, &idx, sub, gsub);
    if (!st.ok()) return st;
  }
  *next = idx;
  return Status::Ok();
}

Status OpenFile(const uint8_t *buf, int64_t len, FileMeta *out) {
  *out = FileMeta();
  if (len < 4) return Status::Err(PQ_ERR_EOF, "read the file magic header failed");
  if (memcmp(buf, "PAR1", 4) != 0) return Status::Err(PQ_ERR_INVALID, "invalid parquet file header");
  if (len < 8 || memcmp(buf + len - 4, "PAR1", 4) != 0) return Status::Err(PQ_ERR_INVALID, "invalid parquet file footer");
  int32_t fl;
  memcpy(&fl, buf + len - 8, 4);
  if (fl <= 0) return Status::Err(PQ_ERR_INVALID, "invalid footer len");
  int64_t start = len - 8 - (int64_t)fl;
  if (start < 0) return Status::Err(PQ_ERR_INVALID, "seek file meta data failed");
  ThriftReader t(buf + start, fl);
  int16_t last = 0, id;
  int ty;
  unsigned set = 0;
  while (t.field(&last, &id, &ty)) {
    if (id == 1 && ty == CT_I32) { t.i32(); set |= 1; }
    else if (id == 2 && ty == CT_LIST) {
      read_struct_list(t, &out->schema, read_schema_element, fl);
      set |= 2;
    } else if (id == 3 && ty == CT_I64) { out->num_rows = t.i64(); set |= 4; }
    else if (id == 4 && ty == CT_LIST) {
      read_struct_list(t, &out->row_groups, [fl](ThriftReader &tt, RowGroup *g) { read_row_group(tt, g, fl); }, fl);
      set |= 8;
    } else skip_field(t, ty);
  }
  if (t.failed() || set != 15) return Status::Err(PQ_ERR_THRIFT, "read file meta failed");
  // makeSchema schema.go:1048-1079: schema[0] is the root.
  if (out->schema.empty()) return Status::Err(PQ_ERR_INVALID, "no schema element found");
  int32_t n = (int32_t)out->schema.size() - 1;
  for (int32_t idx = 0; idx < n;) {
    Status st = !out->schema[1 + (size_t)idx].has_type ? read_group_schema(out, 1, n, idx, "", 0, 0, &idx, 0, {}, {})
                                                      : read_column_schema(out, 1, idx, "", 0, 0, &idx, {}, {});
    if (!st.ok()) return Status::Err(st.code, "creating schema failed: " + st.msg);
  }
  return Status::Ok();
}

// ---------------------------------------------------------------------------
// Host block decompression (compress.go:34-76)
// ---------------------------------------------------------------------------
bool SnappyDecodedLen(const uint8_t *src, int64_t n, int64_t *len) {
  uint64_t v = 0;
  unsigned sh = 0;
  for (int64_t k = 0; k < 10; k++) {
    if (k >= n) return false;
    uint8_t b = src[k];
    if (b < 0x80) {
      if (k == 9 && b > 1) return false;
      v |= (uint64_t)b << sh;
      if (v > 0xffffffffULL) return false;
      *len = (int64_t)v;
      return true;
    }
    v |= (uint64_t)(b & 0x7f) << sh;
    sh += 7;
  }
  return false;
}

// Raw snappy block elements (golang/snappy v0.0.1 decode_other.go:20-96 semantics: any
// inconsistency is ErrCorrupt), resumable so the planner can decode just a page's head.
bool SnappyPrefix::Extend(int64_t want) {
  if (want > dlen) want = dlen;
  while (d < want && s < n) {
    uint8_t tag = src[s];
    int64_t length, offset;
    if ((tag & 3) == 0) {
      uint32_t x = tag >> 2;
      if (x < 60) s += 1;
      else {
        int nb = (int)x - 59;
        if (s + 1 + nb > n) return false;
        x = 0;
        for (int k = 0; k < nb; k++) x |= (uint32_t)src[s + 1 + k] << (8 * k);
        s += 1 + nb;
      }
      length = (int64_t)x + 1;
      if (length > dlen - d || length > n - s) return false;
      memcpy(dst + d, src + s, (size_t)length);
      d += length;
      s += length;
      continue;
    }
    if ((tag & 3) == 1) {
      if (s + 2 > n) return false;
      length = 4 + ((tag >> 2) & 7);
      offset = ((int64_t)(tag & 0xe0) << 3) | src[s + 1];
      s += 2;
    } else if ((tag & 3) == 2) {
      if (s + 3 > n) return false;
      length = 1 + (tag >> 2);
      offset = src[s + 1] | ((int64_t)src[s + 2] << 8);
      s += 3;
    } else {
      if (s + 5 > n) return false;
      length = 1 + (tag >> 2);
      offset = src[s + 1] | ((int64_t)src[s + 2] << 8) | ((int64_t)src[s + 3] << 16) | ((int64_t)src[s + 4] << 24);
      s += 5;
    }
    if (offset <= 0 || d < offset || length > dlen - d) return false;
    if (offset >= length) {
      memcpy(dst + d, dst + d - offset, (size_t)length);
    } else {
      for (int64_t k = 0; k < length; k++) dst[d + k] = dst[d - offset + k];
    }
    d += length;
  }
  return true;
}

bool SnappyPrefix::Init(const uint8_t *block, int64_t len, uint8_t *out, int64_t cap) {
  if (!SnappyDecodedLen(block, len, &dlen)) return false;
  int64_t v = 0;
  while (v < len && (block[v] & 0x80)) v++;
  v++;
  src = block + v;
  n = len - v;
  s = d = 0;
  dst = out;
  return dlen <= cap;
}

Status SnappyDecode(const uint8_t *src, int64_t n, uint8_t *dst, int64_t dst_cap, int64_t *dst_len) {
  SnappyPrefix sp;
  if (!sp.Init(src, n, dst, dst_cap)) return Status::Err(PQ_ERR_DECOMPRESS, "snappy: corrupt input");
  // trailing elements after the last byte would each overflow dst: corrupt
  if (!sp.Extend(sp.dlen) || sp.s != sp.n || sp.d != sp.dlen) return Status::Err(PQ_ERR_DECOMPRESS, "snappy: corrupt input");
  *dst_len = sp.dlen;
  return Status::Ok();
}

static Status gzip_decode(const uint8_t *src, int64_t n, std::vector<uint8_t> *out) {
  size_t base = out->size();
  size_t cap = (size_t)n * 4 + 1024;
  out->resize(base + cap);
  int64_t pos = 0, len = 0;
  int members = 0;
  while (pos < n || members == 0) {
    z_stream zs;
    memset(&zs, 0, sizeof(zs));
    if (inflateInit2(&zs, 16 + MAX_WBITS) != Z_OK) return Status::Err(PQ_ERR_DECOMPRESS, "gzip: init");
    zs.next_in = (Bytef *)(src + pos);
    zs.avail_in = (uInt)(n - pos);
    int rc;
    do {
      if ((size_t)len == cap) {
        cap *= 2;
        out->resize(base + cap);
      }
      zs.next_out = out->data() + base + len;
      zs.avail_out = (uInt)(cap - (size_t)len);
      rc = inflate(&zs, Z_NO_FLUSH);
      len = (int64_t)cap - zs.avail_out;
      if (rc != Z_OK && rc != Z_STREAM_END && !(rc == Z_BUF_ERROR && zs.avail_out == 0)) {
        inflateEnd(&zs);
        out->resize(base);
        return Status::Err(PQ_ERR_DECOMPRESS, "gzip: invalid data");
      }
    } while (rc != Z_STREAM_END);
    pos = n - zs.avail_in;
    inflateEnd(&zs);
    members++;
  }
  out->resize(base + (size_t)len);
  return Status::Ok();
}

Status Decompress(int32_t codec, const uint8_t *src, int64_t n, std::vector<uint8_t> *out) {
  if (codec == 0) {
    out->insert(out->end(), src, src + n);
    return Status::Ok();
  }
  if (codec == 1) {
    int64_t dlen;
    if (!SnappyDecodedLen(src, n, &dlen)) return Status::Err(PQ_ERR_DECOMPRESS, "decompression failed: snappy: corrupt input");
    size_t base = out->size();
    out->resize(base + (size_t)dlen);
    int64_t got;
    Status st = SnappyDecode(src, n, out->data() + base, dlen, &got);
    if (!st.ok()) { out->resize(base); return Status::Err(st.code, "decompression failed: " + st.msg); }
    return Status::Ok();
  }
  if (codec == 2) return gzip_decode(src, n, out);
  return Status::Err(PQ_ERR_UNSUPPORTED, "decompression failed: method is not supported");
}

}  // namespace pq
