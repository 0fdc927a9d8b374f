/*
 * pqgpu.h — C ABI of the MI355X-native Parquet column-chunk decoder.
 *
 * This is the drop-in boundary for the read path of fraugster/parquet-go
 * (v0.12.0 line). Each entry point names the reference interface it
 * replaces (file:line under the reference tree). A Go `gpudecode` package
 * binds these through cgo; the same symbols are bound
 * from Python via ctypes for the parity tests and the benchmark.
 *
 * Conventions
 *  - Plain C types only; no HIP or torch types in signatures. `stream` is a
 *    hipStream_t passed as void* (NULL = the context's own stream).
 *  - Every function returns a pqgpu status (PQ_OK = 0) and, where it takes
 *    a pqgpu_error*, fills it with the error class, the failing chunk/page
 *    and a message mirroring the reference's error text.
 *  - Error classes mirror the Go error values the reference returns; the
 *    numbering is shared with the CPU oracle (oracle/oracle.h).
 *  - Thread safety: one pqgpu_ctx per GPU; a batch is used by one host
 *    thread at a time (the reference FileReader is not goroutine-safe
 *    either, file_reader.go:18); different batches of one ctx may be driven
 *    from different threads on different streams (the pipeline does).
 */
#ifndef PQGPU_H
#define PQGPU_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PQGPU_ABI_VERSION 8

/* Error classes (Go error value the reference returns in the same case). */
enum pqgpu_status {
  PQ_OK = 0,
  PQ_ERR_EOF = 1,            /* io.EOF */
  PQ_ERR_UNEXPECTED_EOF = 2, /* io.ErrUnexpectedEOF */
  PQ_ERR_INVALID = 3,        /* malformed data: errors.New / fmt.Errorf in the decoders */
  PQ_ERR_UNSUPPORTED = 4,    /* unsupported type / encoding / codec */
  PQ_ERR_DICT_INDEX = 5,     /* "dict: invalid index %d, values count are %d" type_dict.go:52-54 */
  PQ_ERR_CRC = 6,            /* "CRC32 check failed" chunk_reader.go:173-177 */
  PQ_ERR_DECOMPRESS = 7,     /* "decompression failed" / size mismatch compress.go:102-123 */
  PQ_ERR_THRIFT = 8,         /* thrift decode error (readThrift helpers.go:103-109) */
  PQ_ERR_RANGE = 9,          /* "int32 out of range" helpers.go:176 / varint overflow */
  PQ_ERR_NOMEM = 10,         /* host or device allocation failure */
  PQ_ERR_ARG = 11,           /* bad argument to this API */
  PQ_ERR_HIP = 12,           /* HIP runtime error (no GPU, launch failure, ...) */
};

/* parquet.Type (parquet/parquet.go) */
enum { PQ_BOOLEAN = 0, PQ_INT32 = 1, PQ_INT64 = 2, PQ_INT96 = 3, PQ_FLOAT = 4, PQ_DOUBLE = 5,
       PQ_BYTE_ARRAY = 6, PQ_FIXED_LEN_BYTE_ARRAY = 7 };

typedef struct {
  int32_t code;     /* enum pqgpu_status */
  int32_t chunk;    /* batch chunk id, -1 if not chunk specific */
  int32_t page;     /* data-page index within the chunk, -1 for chunk-level errors */
  char msg[244];
} pqgpu_error;

typedef struct pqgpu_ctx pqgpu_ctx;
typedef struct pqgpu_file pqgpu_file;
typedef struct pqgpu_batch pqgpu_batch;

/* Leaf column schema: Column.maxD/maxR from readColumnSchema schema.go:893-924. */
typedef struct {
  int32_t physical_type;   /* parquet.Type */
  int32_t type_length;     /* FIXED_LEN_BYTE_ARRAY length */
  int32_t max_def;         /* Column.MaxDefinitionLevel() */
  int32_t max_rep;         /* Column.MaxRepetitionLevel() */
  int32_t repetition;      /* leaf parquet.FieldRepetitionType */
  char path[236];          /* dotted ColumnPath */
  /* Nested (Arrow-style) output, per REPEATED node on the path, outermost first
   * (max_rep entries, at most PQGPU_MAX_NEST): the definition level before the
   * node (the list is non-null from it) and at the node (the list has an
   * element from it). Filled by pqgpu_file_column from the schema. */
  int32_t list_null_def[8];
  int32_t list_def[8];
  /* OPTIONAL groups on the path, outermost first (num_groups <= PQGPU_MAX_NEST;
   * the leaf itself is not one): the group's definition level (it is non-null
   * from it), the REPEATED nodes above it (its entries are the records at 0,
   * else the elements of list level group_depth - 1) and its position in the
   * dotted path (0 = the top-level field). Filled by pqgpu_file_column. */
  int32_t num_groups;
  int32_t group_def[8];
  int32_t group_depth[8];
  int32_t group_node[8];
  int32_t list_node[8];    /* path position of each REPEATED node (list level k) */
} pqgpu_column_info;
#define PQGPU_MAX_NEST 8

/* The subset of parquet.ColumnMetaData that readChunk consults
 * (chunk_reader.go:299-362). Offsets are absolute file offsets. */
typedef struct {
  int32_t physical_type;
  int32_t codec;                   /* parquet.CompressionCodec */
  int64_t num_values;
  int64_t total_compressed_size;
  int64_t data_page_offset;
  int64_t dictionary_page_offset;  /* -1 when unset */
  int32_t has_file_path;           /* ColumnChunk.FilePath != nil -> "nyi" error */
  int32_t pad;
} pqgpu_chunk_meta;

/* Decoded column chunk. Device pointers stay owned by the batch.
 *  values     fixed-width values of the non-null slots, in order (the
 *             reference's []interface{} returned by readValues,
 *             page_v1.go:53 / page_v2.go:51): INT32/FLOAT 4 B, INT64/DOUBLE
 *             8 B, INT96 12 B, BOOLEAN 1 B (0/1), FIXED_LEN_BYTE_ARRAY
 *             type_length B. NULL for BYTE_ARRAY.
 *  offsets    BYTE_ARRAY: int32[num_values+1] into payload.
 *  payload    BYTE_ARRAY bytes.
 *  def_levels uint8 per slot (the reference's dLevel packedArray) when
 *             max_def > 0; NULL otherwise (all levels are 0).
 *  rep_levels uint8 per slot when max_rep > 0, else NULL.
 *  validity   bitmap, bit i (LSB-first) = def_levels[i] == max_def
 *             (Arrow layout); NULL when max_def == 0 (all valid).
 *  list_offsets (max_rep > 0): int32[num_records+1]; record r spans slots
 *             [list_offsets[r], list_offsets[r+1]) — record boundaries are
 *             the slots with rep_level == 0 (ColumnStore.get data_store.go:285-308).
 */
typedef struct {
  int64_t num_slots;
  int64_t num_values;
  int64_t num_records;
  int64_t payload_bytes;
  int32_t physical_type;
  int32_t value_width;
  int32_t max_def;
  int32_t max_rep;
  void *values;
  int32_t *offsets;
  uint8_t *payload;
  uint8_t *def_levels;
  uint8_t *rep_levels;
  uint32_t *validity;
  int32_t *list_offsets;
  /* Nested (Arrow-style) arrays of a repeated leaf (nest_levels = max_rep when
   * max_rep <= PQGPU_MAX_NEST, else 0). List level k (0 = outermost REPEATED
   * node) has num_lists[k] lists; list j spans child entries
   * [lvl_offsets[k][j], lvl_offsets[k][j+1]) — the lists of level k+1, or for
   * the innermost level the leaf's element slots; bit j of lvl_validity[k] =
   * list j is non-null (null and empty lists both have no children). The leaf
   * has num_elements element slots; bit e of element_validity = element e is
   * non-null, and `values` holds the non-null elements in order. */
  int32_t nest_levels;
  int32_t dictionary_page;  /* 1 when the chunk had a dictionary page (readChunk's useDict) */
  int64_t num_lists[8];
  int32_t *lvl_offsets[8];
  uint32_t *lvl_validity[8];
  int64_t num_elements;
  uint32_t *element_validity;
  /* Struct validity of the OPTIONAL groups on the path (column info
   * num_groups / group_*; produced with the nested arrays, and for leaves with
   * max_rep == 0): group g has group_entries[g] entries — the records (for a
   * max_rep == 0 leaf its slots), else the element entries of list level
   * group_depth[g] - 1 — and bit e of group_validity[g] = the group of entry e
   * is non-null. Column.getNextData (schema.go:216-260) makes a group nil
   * unless a child is defined at or below the group's own level, i.e. bit =
   * (def >= group_def[g]). A pointer may alias lvl_validity / element_validity /
   * validity when the bitmaps are equal. */
  int32_t num_groups;
  int32_t pad1;
  int64_t group_entries[8];
  uint32_t *group_validity[8];
} pqgpu_chunk_result;

/* Per-batch statistics, for the roofline accounting. */
typedef struct {
  int64_t num_chunks;
  int64_t num_pages;
  int64_t num_slots;
  int64_t num_values;
  int64_t input_bytes;       /* rep+def+value section bytes (decompressed) + dictionary payloads */
  int64_t output_bytes;      /* values + levels + validity + offsets + payload materialised */
  int64_t staged_bytes;      /* bytes resident in HBM as the decoder's input */
  double host_plan_ms;       /* page-header walk + descriptor build (host) */
  double host_decompress_ms; /* GZIP (and PQ_HOST_SNAPPY=1 SNAPPY) pages on the host */
  int64_t levels_kernel_bytes; /* algorithmic bytes of k_levels: level sections + validity/levels written */
  int64_t values_kernel_bytes; /* algorithmic bytes of k_values: value sections + values/offsets written */
  int64_t delta_kernel_bytes;  /* the DELTA_BINARY_PACKED pages' share of values_kernel_bytes */
  int64_t snappy_pages;        /* SNAPPY data pages decompressed on the device (k_snappy) */
  int64_t snappy_kernel_bytes; /* algorithmic bytes of k_snappy: blocks + raw level bytes read, pages written */
} pqgpu_batch_stats;

/* ---- version / device ---------------------------------------------- */
int pqgpu_abi_version(void);
const char *pqgpu_status_string(int code);

/* One context per GPU. Replaces the per-FileReader decode state. */
int pqgpu_ctx_create(int device, pqgpu_ctx **out, pqgpu_error *err);
void pqgpu_ctx_destroy(pqgpu_ctx *ctx);

/* ---- file metadata (host) ------------------------------------------- */
/* ReadFileMetaData(r, true) + makeSchema: file_meta.go:24-74,
 * schema.go:1048-1079. `buf` is borrowed and must outlive the file. */
int pqgpu_file_open(const uint8_t *buf, size_t len, pqgpu_file **out, pqgpu_error *err);
void pqgpu_file_close(pqgpu_file *f);
int pqgpu_file_num_row_groups(const pqgpu_file *f);
/* The borrowed file buffer passed to pqgpu_file_open, and its length. */
const uint8_t *pqgpu_file_bytes(const pqgpu_file *f);
size_t pqgpu_file_len(const pqgpu_file *f);
int pqgpu_file_num_columns(const pqgpu_file *f);
int64_t pqgpu_file_row_group_num_rows(const pqgpu_file *f, int rg);
int pqgpu_file_column(const pqgpu_file *f, int col, pqgpu_column_info *out);
int pqgpu_file_chunk_meta(const pqgpu_file *f, int rg, int col, pqgpu_chunk_meta *out, pqgpu_error *err);

/* ---- batched chunk decode ------------------------------------------- */
/* ctx may be NULL: a plan-only batch that walks and validates page headers
 * (add_chunk) without a GPU; upload/decode then fail with PQ_ERR_HIP. */
int pqgpu_batch_create(pqgpu_ctx *ctx, pqgpu_batch **out, pqgpu_error *err);
void pqgpu_batch_destroy(pqgpu_batch *b);
/* Drop all chunks (keeps device allocations for reuse). */
int pqgpu_batch_reset(pqgpu_batch *b);

/* readChunk + readPages (chunk_reader.go:182-362): walk the chunk's page
 * headers on the host, validate them exactly as the reference does, and
 * stage the page sections for upload. GZIP pages (and dictionary pages) are
 * decompressed on the host; SNAPPY data pages are staged compressed and
 * decompressed by k_snappy at the start of every decode (the host decodes
 * only the page head it validates; PQ_HOST_SNAPPY=1 forces host decoding).
 * A corrupt SNAPPY block is reported at sync as that page's PQ_ERR_DECOMPRESS,
 * in the reference's order (compress.go:102-123). `file_bytes` is the whole file (offsets in `meta`
 * are absolute); `col` carries maxD/maxR (schema.go:893-924).
 * A chunk-level error is recorded and returned here; the chunk id is still
 * assigned so its error can be queried later. */
int pqgpu_batch_add_chunk(pqgpu_batch *b, const uint8_t *file_bytes, size_t file_len,
                          const pqgpu_column_info *col, const pqgpu_chunk_meta *meta,
                          int validate_crc, int32_t *chunk_id, pqgpu_error *err);
/* Convenience: column `col` of row group `rg` of an opened file
 * (FileReader.readRowGroupData chunk_reader.go:375-404). */
int pqgpu_batch_add_file_chunk(pqgpu_batch *b, const pqgpu_file *f, int rg, int col, int validate_crc,
                               int32_t *chunk_id, pqgpu_error *err);

/* ---- on-device page index -------------------
 * readPages' page-header loop (chunk_reader.go:182-263), the Thrift compact
 * decode of every PageHeader (readThrift helpers.go:103-109) and readPageBlock's
 * CRC32 check (chunk_reader.go:173-177), on the GPU, for column chunks whose
 * bytes are resident in device memory: `dev_bytes` (16-byte aligned) holds
 * file bytes [file_offset, file_offset + len), e.g. one row group's byte
 * range copied H2D once. One wavefront per chunk walks the header chain;
 * with validate_crc every checksummed block is checked by k_page_crc. The
 * walk takes the valid case only: a chunk it cannot take (a Thrift error, a
 * negative size, a block past the resident bytes) is marked
 * PQGPU_IX_FALLBACK and pqgpu_batch_add_indexed_chunk walks it on the host,
 * so every error keeps the reference's class, message and page. Synchronous
 * (the page table is read back). */
typedef struct pqgpu_page_index pqgpu_page_index;
enum { PQGPU_IX_OK = 0, PQGPU_IX_FALLBACK = 1 };
/* PageHeader flags */
enum { PQGPU_PH_CRC = 1, PQGPU_PH_DATA_PAGE = 2, PQGPU_PH_DICTIONARY_PAGE = 4, PQGPU_PH_DATA_PAGE_V2 = 8,
       PQGPU_PH_V2_COMPRESSED = 16, PQGPU_PH_CRC_CHECKED = 32, PQGPU_PH_CRC_OK = 64 };
typedef struct {
  int64_t header_offset;          /* file offset of the PageHeader */
  int32_t header_len;             /* its Thrift bytes */
  int32_t type;                   /* parquet.PageType */
  int32_t uncompressed_page_size;
  int32_t compressed_page_size;
  int32_t crc;
  int32_t flags;                  /* PQGPU_PH_* (which optional members are set) */
  int32_t data_page[4];           /* DataPageHeader: num_values, encoding, def/rep level encoding */
  int32_t dictionary_page[2];     /* DictionaryPageHeader: num_values, encoding */
  int32_t data_page_v2[6];        /* DataPageHeaderV2: num_values, num_nulls, num_rows, encoding,
                                     definition / repetition levels byte length */
} pqgpu_page_header;
int pqgpu_page_index_build(pqgpu_ctx *ctx, const void *dev_bytes, int64_t file_offset, int64_t len,
                           const pqgpu_chunk_meta *metas, int32_t n_chunks, int32_t validate_crc, void *stream,
                           pqgpu_page_index **out, pqgpu_error *err);
int pqgpu_page_index_chunk(const pqgpu_page_index *ix, int32_t chunk, int32_t *num_pages, int32_t *status);
int pqgpu_page_index_page(const pqgpu_page_index *ix, int32_t chunk, int32_t k, pqgpu_page_header *out);
double pqgpu_page_index_walk_ms(const pqgpu_page_index *ix);
/* How the build went: result read-backs beyond the first (some chunk's completion marker, a
 * per-build generation, was not yet visible), chunks that never reported (walked by the host),
 * chunks that fell back for any reason, 1 when the header table overflowed its largest size
 * (every chunk then falls back), and table entries dropped because they carry another build's
 * generation stamp (left in reused scratch; their chunk's count no longer adds up, so the host
 * walks it). Any pointer may be NULL. */
int pqgpu_page_index_stats(const pqgpu_page_index *ix, int32_t *polls, int32_t *unreported, int32_t *fallback_chunks,
                           int32_t *overflowed, int32_t *stale_entries);
void pqgpu_page_index_destroy(pqgpu_page_index *ix);
/* The host's PageHeader decode (the same fields), for comparison. */
int pqgpu_parse_page_header(const uint8_t *buf, size_t len, pqgpu_page_header *out, int64_t *consumed);
/* pqgpu_batch_add_chunk for chunk `ix_chunk` of an index (its chunk meta): the
 * page headers and CRC verdicts come from the device walk, and UNCOMPRESSED
 * data pages are not copied on the host — their blocks are copied device to
 * device from the resident bytes at upload (k_page_gather), so `dev_bytes`
 * must stay valid until pqgpu_batch_upload returns. `file_bytes` (host) is
 * still read for page heads (V1 level lengths, value-decoder headers),
 * dictionary and compressed pages, and for chunks that fell back. */
int pqgpu_batch_add_indexed_chunk(pqgpu_batch *b, const pqgpu_page_index *ix, int32_t ix_chunk,
                                  const uint8_t *file_bytes, size_t file_len, const pqgpu_column_info *col,
                                  int validate_crc, int32_t *chunk_id, pqgpu_error *err);
int pqgpu_batch_add_indexed_file_chunk(pqgpu_batch *b, const pqgpu_page_index *ix, int32_t ix_chunk,
                                       const pqgpu_file *f, int col, int validate_crc, int32_t *chunk_id,
                                       pqgpu_error *err);

/* Copy staged page bytes and descriptors to HBM (hipMemcpyAsync from
 * pinned memory) and allocate the outputs. */
int pqgpu_batch_upload(pqgpu_batch *b, void *stream, pqgpu_error *err);
/* Launch the decode kernels (pageReader.readValues for every page of every
 * chunk, page_v1.go:33-63 / page_v2.go:31-60). Asynchronous except for
 * BYTE_ARRAY dictionary chunks, whose payload size is read back once. */
int pqgpu_batch_decode(pqgpu_batch *b, void *stream, pqgpu_error *err);
/* Wait for the batch and return the first error in (chunk, page, stage)
 * order — the error the reference's readValues would have returned. */
int pqgpu_batch_sync(pqgpu_batch *b, void *stream, pqgpu_error *err);
/* Wait for the batch's decodes to finish on the device, without collecting
 * their errors or counts (pqgpu_batch_sync does both; results and status are
 * valid only after it). A timing boundary: the decode work is done when it
 * returns. A hipError_t failure is returned as PQ_ERR_HIP. */
int pqgpu_batch_wait(pqgpu_batch *b, void *stream, pqgpu_error *err);

int pqgpu_batch_num_chunks(const pqgpu_batch *b);
/* Per-chunk status after sync (the error of that chunk alone). */
int pqgpu_batch_chunk_status(const pqgpu_batch *b, int32_t chunk_id, pqgpu_error *err);
/* A failed chunk returns its error; when the failure is a page's readValues
 * error (err->page >= 0, not a decompression or CRC error, which the
 * reference raises in readPages before any value is read), *out still
 * describes the decoded pages before the failing page — the rows the
 * reference's lazy page reader returns before it fails (data_store.go:236-260).
 * Otherwise *out is zeroed. */
int pqgpu_batch_chunk_result(const pqgpu_batch *b, int32_t chunk_id, pqgpu_chunk_result *out, pqgpu_error *err);
/* Per-page split of a decoded chunk, the reference's pageReader granularity
 * (ColumnStore.readNextPage data_store.go:236-260 reads one page at a time):
 * data page k of the chunk owns level slots [slot_first[k], +slot_count[k])
 * and non-null values [value_first[k], +value_count[k]) of the chunk result.
 * Call with cap = 0 to query *num_pages. Valid after pqgpu_batch_sync. A
 * chunk error's pqgpu_error.page names the page whose readValues fails. */
int pqgpu_batch_chunk_pages(const pqgpu_batch *b, int32_t chunk_id, int32_t *num_pages, int64_t *slot_first,
                            int64_t *slot_count, int64_t *value_first, int64_t *value_count, int32_t cap,
                            pqgpu_error *err);
/* Copy one chunk's outputs to host buffers sized from pqgpu_batch_chunk_result
 * (any pointer may be NULL to skip that array); for a chunk that failed in a
 * page, the pages before it are copied and the error is returned. */
int pqgpu_batch_copy_chunk(const pqgpu_batch *b, int32_t chunk_id, void *values, int32_t *offsets, uint8_t *payload,
                           uint8_t *def_levels, uint8_t *rep_levels, uint32_t *validity, int32_t *list_offsets,
                           pqgpu_error *err);
/* Copy list level `level`'s offsets (num_lists + 1) and validity words, and
 * the element validity words, of a nested chunk to host buffers (any may be NULL). */
int pqgpu_batch_copy_nested(const pqgpu_batch *b, int32_t chunk_id, int32_t level, int32_t *offsets,
                            uint32_t *validity, uint32_t *element_validity, pqgpu_error *err);
/* Copy group g's struct validity words ((group_entries[g] + 31) / 32) to a host buffer. */
int pqgpu_batch_copy_group(const pqgpu_batch *b, int32_t chunk_id, int32_t group, uint32_t *validity, pqgpu_error *err);
/* Two leaves of one group — a MAP's key and value, or sibling fields of a
 * struct (Column.getNextData reads every child of a group at the same
 * position, schema.go:216-312): the nested arrays of their common ancestors
 * (the list levels and OPTIONAL groups on the shared path prefix) must be
 * identical. They are compared on the device; when equal, *equal = 1 and
 * chunk_b's result carries chunk_a's arrays for those levels and groups (one
 * shared offsets array per list level, one bitmap per group) until the next
 * decode; otherwise *equal = 0 and nothing changes. Both chunks must have
 * decoded without error; PQ_ERR_ARG when their paths share no ancestor
 * structure consistently (e.g. leaves of different files). */
int pqgpu_batch_share_ancestors(pqgpu_batch *b, int32_t chunk_a, int32_t chunk_b, int32_t *equal, pqgpu_error *err);
int pqgpu_batch_stats_get(const pqgpu_batch *b, pqgpu_batch_stats *out);
/* Diagnostics: 64 device counters filled by in-kernel phase stamps when the
 * environment has PQ_DEBUG_STAMPS=1 at upload time. */
int pqgpu_batch_debug_counters(pqgpu_batch *b, uint64_t *out64, int reset);

/* Timing hook for the benchmark: average duration (ms) of the dominant
 * decode kernel over the last `pqgpu_batch_decode` calls, measured with HIP
 * events on the stream the kernel runs on; and its name. */
int pqgpu_batch_kernel_timing(pqgpu_batch *b, int enable);
int pqgpu_batch_kernel_time(pqgpu_batch *b, double *avg_ms, int64_t *launches, char *name, size_t name_len);
/* The same for every timed launch slot (0 <= slot < PQGPU_TIMER_SLOTS); PQ_ERR_ARG past the end. */
#define PQGPU_TIMER_SLOTS 25
int pqgpu_batch_kernel_slot(pqgpu_batch *b, int slot, double *avg_ms, int64_t *launches, char *name,
                            size_t name_len);
/* Algorithmic bytes (sections read + outputs written, counted once) of one launch
 * of timer slot `slot` for the last synced decode: the roofline numerator of that kernel. */
int pqgpu_batch_kernel_bytes(const pqgpu_batch *b, int slot, int64_t *bytes);

/* Device-to-device (or host) copy on the library's own HIP runtime, for
 * callers that hold device pointers of a chunk result, e.g. when gathering
 * a row-group shard into one column: hipMemcpy, hipMemcpyDefault. */
int pqgpu_copy(pqgpu_ctx *ctx, void *dst, const void *src, size_t bytes, pqgpu_error *err);
/* Device memory on the library's runtime (hipMalloc, 256-byte aligned), e.g. for
 * file bytes made resident for pqgpu_page_index_build (copy them with pqgpu_copy). */
int pqgpu_dev_alloc(pqgpu_ctx *ctx, size_t bytes, void **out, pqgpu_error *err);
void pqgpu_dev_free(pqgpu_ctx *ctx, void *p);

/* ---- streaming row-group pipeline -------------------------------------
 * FileReader.readRowGroupData (chunk_reader.go:375-404) called for row group
 * after row group (file_reader.go:187-198), as a stream: host worker threads
 * plan row group k + 1 .. k + depth - 1 (page-header walk, GZIP and
 * dictionary pages, pinned staging) and enqueue its H2D copy and decode on
 * its own stream while the GPU decodes row group k. Each row group is one
 * batch holding the requested columns; batches come back in row-group order. */
typedef struct pqgpu_pipeline pqgpu_pipeline;
typedef struct {
  int32_t depth;         /* row groups in flight (batches); >= 2 double-buffers, default 3 */
  int32_t threads;       /* host planner threads; 0 = depth */
  int32_t validate_crc;  /* WithCRC32Validation (file_reader.go:134-139) */
  int32_t device_index;  /* 1: each row group's byte range is copied to the device once and its page
                            headers walked (and checksummed) there (pqgpu_page_index_build);
                            UNCOMPRESSED page bodies then reach the decoder device to device */
} pqgpu_pipeline_opts;
typedef struct {
  int64_t row_groups;      /* row groups returned so far */
  int64_t rows;
  int64_t chunks;
  int64_t failed_chunks;
  int64_t input_bytes;     /* staged page bytes uploaded (H2D) */
  int64_t output_bytes;    /* decoded bytes materialised */
  double wall_ms;          /* pipeline create .. last row group returned */
  double plan_ms;          /* host page-header walks + staging, summed over threads */
  double upload_ms;        /* host side of pqgpu_batch_upload (descriptors, pinned copy), summed */
  double h2d_ms;           /* GPU: upload enqueue .. done, summed over row groups */
  double decode_ms;        /* GPU: decode launches .. done, summed over row groups */
  double index_ms;         /* device_index: byte-range copy + device page walk, summed (part of plan_ms) */
  /* device_index builds (pqgpu_page_index_stats summed): result re-reads, chunks whose walk never
   * reported (walked by the host), chunks the host walked for any reason, stale table entries dropped */
  int64_t ix_polls, ix_unreported, ix_fallback_chunks, ix_stale_entries;
} pqgpu_pipeline_stats;
/* rgs / cols may be NULL for all row groups / all columns. */
int pqgpu_pipeline_create(pqgpu_ctx *ctx, const pqgpu_file *f, const int32_t *rgs, int32_t n_rgs, const int32_t *cols,
                          int32_t n_cols, const pqgpu_pipeline_opts *opts, pqgpu_pipeline **out, pqgpu_error *err);
/* The next row group, decoded and synced: *batch holds its chunks (column
 * order of `cols`), *rg its index; the batch stays valid until
 * pqgpu_pipeline_release. At the end *batch is NULL and PQ_OK is returned.
 * The return value is the batch's first chunk error (as pqgpu_batch_sync). */
int pqgpu_pipeline_next(pqgpu_pipeline *p, pqgpu_batch **batch, int32_t *rg, pqgpu_error *err);
int pqgpu_pipeline_release(pqgpu_pipeline *p, pqgpu_batch *batch);
int pqgpu_pipeline_stats_get(const pqgpu_pipeline *p, pqgpu_pipeline_stats *out);
void pqgpu_pipeline_destroy(pqgpu_pipeline *p);

#ifdef __cplusplus
}
#endif
#endif
