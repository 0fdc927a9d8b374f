/*
 * oracle.h — CPU restatement of fraugster/parquet-go's column-chunk read path.
 *
 * TEST INFRASTRUCTURE ONLY. This library is the parity checker for the
 * MI355X decoder (libpqgpu). Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it. The product path never links,
 * loads or calls anything under oracle/.
 *
 * Every decoder in oracle.c is a value-at-a-time restatement of the Go code
 * it cites (file:line under the reference tree), including its quirks
 * (SURVEY.md Appendix A). Error classes follow the Go error values the
 * reference returns (io.EOF, io.ErrUnexpectedEOF, fmt.Errorf, ...).
 */
#ifndef PQ_ORACLE_H
#define PQ_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Error classes — identical numbering to include/pqgpu.h PQ_ERR_*. */
enum {
  OR_OK = 0,
  OR_ERR_EOF = 1,            /* io.EOF */
  OR_ERR_UNEXPECTED_EOF = 2, /* io.ErrUnexpectedEOF */
  OR_ERR_INVALID = 3,        /* malformed data (errors.New / fmt.Errorf) */
  OR_ERR_UNSUPPORTED = 4,    /* unsupported type/encoding/codec */
  OR_ERR_DICT_INDEX = 5,     /* dict: invalid index */
  OR_ERR_CRC = 6,            /* CRC32 check failed */
  OR_ERR_DECOMPRESS = 7,     /* decompression failed / size mismatch */
  OR_ERR_THRIFT = 8,         /* thrift decode error */
  OR_ERR_RANGE = 9,          /* int32 out of range / varint overflow */
  OR_ERR_NOMEM = 10,
  OR_ERR_ARG = 11,
};

typedef struct or_file or_file;

typedef struct {
  int32_t physical_type; /* parquet.Type */
  int32_t type_length;   /* FIXED_LEN_BYTE_ARRAY length, else 0 */
  int32_t max_def;
  int32_t max_rep;
  int32_t repetition;    /* leaf FieldRepetitionType */
  char path[256];        /* dotted path */
  int32_t path_len;      /* nodes on the path (groups, then the leaf) */
  int32_t node_rep[64];  /* FieldRepetitionType of each node on the path (nested-array checks) */
} or_column_info;

typedef struct {
  int32_t err_code;
  int32_t err_page;       /* index of the data page that failed (-1: chunk level) */
  char err_msg[256];
  int64_t num_slots;      /* number of (rep, def) level slots */
  int64_t num_values;     /* number of non-null values (def == maxD) */
  int32_t value_width;    /* bytes per value for fixed width, 0 for byte arrays */
  int32_t num_pages;
  int32_t *def_levels;    /* num_slots */
  int32_t *rep_levels;    /* num_slots */
  uint8_t *values;        /* fixed width: num_values*width; byte arrays: payload */
  int64_t values_bytes;
  int64_t *offsets;       /* byte arrays: num_values+1, else NULL */
} or_chunk_result;

int or_file_open(const uint8_t *buf, size_t len, or_file **out, char *err, size_t errlen);
void or_file_close(or_file *f);
int or_file_num_row_groups(const or_file *f);
int or_file_num_columns(const or_file *f);
int64_t or_file_row_group_num_rows(const or_file *f, int rg);
int or_file_column_info(const or_file *f, int col, or_column_info *out);

/* readChunk + readValues(numValues) for every page of one column chunk. */
int or_read_chunk(const or_file *f, int rg, int col, int validate_crc, or_chunk_result *out);
void or_chunk_result_free(or_chunk_result *r);

/* Codec-level entry points used by the known-answer tests. */
void or_unpack8_int32(const uint8_t *data, int bw, int32_t out[8]);
void or_unpack8_int64(const uint8_t *data, int bw, int64_t out[8]);
/* Hybrid decode of n values from a raw stream (no length prefix). Returns err class. */
int or_hybrid_decode(const uint8_t *buf, size_t len, int bw, int64_t n, int32_t *out, int64_t *decoded);
/* DELTA_BINARY_PACKED decode of up to n values (64-bit). Returns err class. */
int or_delta_decode64(const uint8_t *buf, size_t len, int64_t n, int64_t *out, int64_t *decoded);
int or_delta_decode32(const uint8_t *buf, size_t len, int64_t n, int32_t *out, int64_t *decoded);

#ifdef __cplusplus
}
#endif
#endif
