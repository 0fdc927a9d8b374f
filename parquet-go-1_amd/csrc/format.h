// format.h — host-side Parquet metadata for the MI355X decoder:
// Thrift compact-protocol reader, FileMetaData/PageHeader structs, schema
// levels, host block decompression. Mirrors what the reference reads with
// its generated Thrift code (parquet/parquet.go) and schema.go.
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

namespace pq {

// Error raised while parsing / planning; code is a pqgpu_status.
struct Status {
  int code = 0;
  std::string msg;
  bool ok() const { return code == 0; }
  static Status Ok() { return Status(); }
  static Status Err(int c, std::string m) {
    Status s;
    s.code = c;
    s.msg = std::move(m);
    return s;
  }
};

// Compact-protocol cursor over a byte range (thrift v0.15.0 TCompactProtocol).
class ThriftReader {
 public:
  ThriftReader(const uint8_t *p, int64_t n) : p_(p), n_(n) {}
  int64_t pos() const { return i_; }
  bool failed() const { return err_; }
  bool byte(uint8_t *b);
  uint64_t uvarint();
  int32_t i32() { uint32_t u = (uint32_t)uvarint(); return (int32_t)(u >> 1) ^ -(int32_t)(u & 1); }
  int64_t i64() { uint64_t u = uvarint(); return (int64_t)(u >> 1) ^ -(int64_t)(u & 1); }
  bool binary(std::string *out);  // nullptr -> skip
  bool list_begin(int *etype, int32_t *size);
  // Iterate struct fields: returns false at STOP (or error).
  bool field(int16_t *last, int16_t *id, int *type);
  void skip(int type, int depth = 0);
  void fail() { err_ = true; }

 private:
  const uint8_t *p_;
  int64_t n_, i_ = 0;
  bool err_ = false;
};

struct DataPageHeader { int32_t num_values = 0, encoding = 0, def_enc = 0, rep_enc = 0; };
struct DictPageHeader { int32_t num_values = 0, encoding = 0; };
struct DataPageHeaderV2 {
  int32_t num_values = 0, num_nulls = 0, num_rows = 0, encoding = 0, def_len = 0, rep_len = 0;
  bool is_compressed = true;
};
struct PageHeader {
  int32_t type = 0, usize = 0, csize = 0, crc = 0;
  bool has_crc = false, has_dph = false, has_dict = false, has_dph2 = false;
  DataPageHeader dph;
  DictPageHeader dict;
  DataPageHeaderV2 dph2;
};
// Parse one PageHeader at p; *consumed = header bytes. Returns false on a thrift error.
bool ParsePageHeader(const uint8_t *p, int64_t n, PageHeader *h, int64_t *consumed);

struct SchemaElement {
  bool has_type = false, has_type_length = false, has_rep = false, has_num_children = false;
  int32_t type = 0, type_length = 0, rep = 0, num_children = 0;
  std::string name;
};
struct ColumnChunkMeta {
  bool has_meta = false, has_file_path = false, has_dict_offset = false;
  int32_t type = 0, codec = 0;
  int64_t num_values = 0, total_uncompressed = 0, total_compressed = 0, data_page_offset = 0, dict_offset = 0;
};
struct RowGroup {
  std::vector<ColumnChunkMeta> cols;
  int64_t num_rows = 0;
};
struct Leaf {
  int32_t type = 0, type_length = 0, max_def = 0, max_rep = 0, rep = 0;
  std::string path;
  // per REPEATED node on the path, outermost first (max_rep entries): the definition level
  // before the node (a list at that level is non-null from here) and at the node (it has
  // an element from here)
  std::vector<int32_t> list_null_def, list_def, list_node;  // + the node's position on the dotted path
  // per OPTIONAL group on the path, outermost first: its definition level (the group is non-null
  // from here), the REPEATED nodes above it (its entries are those of that list depth) and its
  // position on the dotted path
  std::vector<int32_t> group_def, group_depth, group_node;
};
struct FileMeta {
  std::vector<SchemaElement> schema;
  std::vector<RowGroup> row_groups;
  std::vector<Leaf> leaves;
  int64_t num_rows = 0;
};

// ReadFileMetaData(r, true) + makeSchema (file_meta.go:24-74, schema.go:893-1079).
Status OpenFile(const uint8_t *buf, int64_t len, FileMeta *out);

// Block decompression (compress.go:34-76): codec 0 copy, 1 snappy, 2 gzip.
// Appends the decoded bytes to *out. Returns PQ_ERR_DECOMPRESS / UNSUPPORTED.
Status Decompress(int32_t codec, const uint8_t *src, int64_t n, std::vector<uint8_t> *out);
Status SnappyDecode(const uint8_t *src, int64_t n, uint8_t *dst, int64_t dst_cap, int64_t *dst_len);
bool SnappyDecodedLen(const uint8_t *src, int64_t n, int64_t *len);
// Resumable decode of a raw snappy block's leading bytes: the planner reads page headers,
// level lengths and value-decoder headers from them while the device decompresses the page.
struct SnappyPrefix {
  const uint8_t *src = nullptr;  // elements (after the length preamble)
  int64_t n = 0, s = 0;          // element bytes, next element
  uint8_t *dst = nullptr;
  int64_t dlen = 0, d = 0;       // decoded length (preamble), bytes decoded so far
  // Parse the preamble; false if it is corrupt or dlen > cap.
  bool Init(const uint8_t *block, int64_t len, uint8_t *out, int64_t cap);
  // Decode whole elements until d >= want (or the end of the elements). false: corrupt.
  bool Extend(int64_t want);
};

}  // namespace pq
