"""pqgpu — Python mirror of parquet-go's read path over the MI355X decoder.

Binds the C ABI in include/pqgpu.h (libpqgpu.so, built in-tree by
`make -C parquet-go-1_amd`) with ctypes and mirrors the reference's reader
interface for the decode path:

    reference (Go, package goparquet)              here
    ------------------------------------------    ---------------------------------
    NewFileReader(r, columns...)  file_reader.go:154   NewFileReader(data, *columns)
    FileReader.NumRowGroups / NumRows                  FileReader.NumRowGroups / NumRows
    FileReader.readRowGroupData  chunk_reader.go:375   FileReader.ReadRowGroupData(rg)
    readChunk + pageReader.readValues (every page)     -> ColumnData per selected leaf
    ColumnStore dLevels / rLevels packedArray          ColumnData.dLevels / rLevels
    []interface{} values (non-null only)               ColumnData.values (ndarray / list of bytes)

Errors are raised as DecodeError carrying the reference's error class
(io.EOF, io.ErrUnexpectedEOF, ...) and the failing page, like
readValues' "read values from page failed" wrapping (page_v1.go:57).

There is no CPU fallback: every decode runs on the GPU; without a GPU (or
without libpqgpu.so) the constructors raise.
"""
import atexit
import ctypes
import os
import weakref

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_PKG = os.path.dirname(_HERE)
LIB_PATH = os.environ.get("PQGPU_LIB") or os.path.join(_PKG, "lib", "libpqgpu.so")  # PQGPU_LIB: diagnostic build

# Error classes (include/pqgpu.h)
PQ_OK, PQ_ERR_EOF, PQ_ERR_UNEXPECTED_EOF, PQ_ERR_INVALID, PQ_ERR_UNSUPPORTED, PQ_ERR_DICT_INDEX = 0, 1, 2, 3, 4, 5
PQ_ERR_CRC, PQ_ERR_DECOMPRESS, PQ_ERR_THRIFT, PQ_ERR_RANGE, PQ_ERR_NOMEM, PQ_ERR_ARG, PQ_ERR_HIP = 6, 7, 8, 9, 10, 11, 12
ERROR_NAMES = {0: "ok", 1: "io.EOF", 2: "io.ErrUnexpectedEOF", 3: "invalid", 4: "unsupported", 5: "dict index",
               6: "crc", 7: "decompress", 8: "thrift", 9: "range", 10: "nomem", 11: "arg", 12: "hip"}

# parquet.Type
BOOLEAN, INT32, INT64, INT96, FLOAT, DOUBLE, BYTE_ARRAY, FIXED_LEN_BYTE_ARRAY = range(8)
_DTYPES = {BOOLEAN: np.uint8, INT32: np.int32, INT64: np.int64, FLOAT: np.uint32, DOUBLE: np.uint64}


class Error(ctypes.Structure):
    _fields_ = [("code", ctypes.c_int32), ("chunk", ctypes.c_int32), ("page", ctypes.c_int32),
                ("msg", ctypes.c_char * 244)]


class ColumnInfo(ctypes.Structure):
    _fields_ = [("physical_type", ctypes.c_int32), ("type_length", ctypes.c_int32), ("max_def", ctypes.c_int32),
                ("max_rep", ctypes.c_int32), ("repetition", ctypes.c_int32), ("path", ctypes.c_char * 236),
                ("list_null_def", ctypes.c_int32 * 8), ("list_def", ctypes.c_int32 * 8),
                ("num_groups", ctypes.c_int32), ("group_def", ctypes.c_int32 * 8), ("group_depth", ctypes.c_int32 * 8),
                ("group_node", ctypes.c_int32 * 8), ("list_node", ctypes.c_int32 * 8)]


class ChunkMeta(ctypes.Structure):
    _fields_ = [("physical_type", ctypes.c_int32), ("codec", ctypes.c_int32), ("num_values", ctypes.c_int64),
                ("total_compressed_size", ctypes.c_int64), ("data_page_offset", ctypes.c_int64),
                ("dictionary_page_offset", ctypes.c_int64), ("has_file_path", ctypes.c_int32),
                ("pad", ctypes.c_int32)]


class ChunkResult(ctypes.Structure):
    _fields_ = [("num_slots", ctypes.c_int64), ("num_values", ctypes.c_int64), ("num_records", ctypes.c_int64),
                ("payload_bytes", ctypes.c_int64), ("physical_type", ctypes.c_int32),
                ("value_width", ctypes.c_int32), ("max_def", ctypes.c_int32), ("max_rep", ctypes.c_int32),
                ("values", ctypes.c_void_p), ("offsets", ctypes.c_void_p), ("payload", ctypes.c_void_p),
                ("def_levels", ctypes.c_void_p), ("rep_levels", ctypes.c_void_p), ("validity", ctypes.c_void_p),
                ("list_offsets", ctypes.c_void_p), ("nest_levels", ctypes.c_int32), ("dictionary_page", ctypes.c_int32),
                ("num_lists", ctypes.c_int64 * 8), ("lvl_offsets", ctypes.c_void_p * 8),
                ("lvl_validity", ctypes.c_void_p * 8), ("num_elements", ctypes.c_int64),
                ("element_validity", ctypes.c_void_p), ("num_groups", ctypes.c_int32), ("pad1", ctypes.c_int32),
                ("group_entries", ctypes.c_int64 * 8), ("group_validity", ctypes.c_void_p * 8)]


class BatchStats(ctypes.Structure):
    _fields_ = [("num_chunks", ctypes.c_int64), ("num_pages", ctypes.c_int64), ("num_slots", ctypes.c_int64),
                ("num_values", ctypes.c_int64), ("input_bytes", ctypes.c_int64), ("output_bytes", ctypes.c_int64),
                ("staged_bytes", ctypes.c_int64), ("host_plan_ms", ctypes.c_double),
                ("host_decompress_ms", ctypes.c_double), ("levels_kernel_bytes", ctypes.c_int64),
                ("values_kernel_bytes", ctypes.c_int64), ("delta_kernel_bytes", ctypes.c_int64),
                ("snappy_pages", ctypes.c_int64), ("snappy_kernel_bytes", ctypes.c_int64)]


class PageHeader(ctypes.Structure):
    """pqgpu_page_header: one PageHeader as the on-device walk (or the host) decoded it."""
    _fields_ = [("header_offset", ctypes.c_int64), ("header_len", ctypes.c_int32), ("type", ctypes.c_int32),
                ("uncompressed_page_size", ctypes.c_int32), ("compressed_page_size", ctypes.c_int32),
                ("crc", ctypes.c_int32), ("flags", ctypes.c_int32), ("data_page", ctypes.c_int32 * 4),
                ("dictionary_page", ctypes.c_int32 * 2), ("data_page_v2", ctypes.c_int32 * 6)]

    def key(self):
        """Every decoded field (flags without the CRC verdict bits), for comparisons."""
        return (self.header_len, self.type, self.uncompressed_page_size, self.compressed_page_size, self.crc,
                self.flags & 31, tuple(self.data_page), tuple(self.dictionary_page), tuple(self.data_page_v2))


PH_CRC, PH_CRC_CHECKED, PH_CRC_OK = 1, 32, 64
IX_OK, IX_FALLBACK = 0, 1


class PipelineOpts(ctypes.Structure):
    _fields_ = [("depth", ctypes.c_int32), ("threads", ctypes.c_int32), ("validate_crc", ctypes.c_int32),
                ("device_index", ctypes.c_int32)]


class PipelineStats(ctypes.Structure):
    _fields_ = [("row_groups", ctypes.c_int64), ("rows", ctypes.c_int64), ("chunks", ctypes.c_int64),
                ("failed_chunks", ctypes.c_int64), ("input_bytes", ctypes.c_int64), ("output_bytes", ctypes.c_int64),
                ("wall_ms", ctypes.c_double), ("plan_ms", ctypes.c_double), ("upload_ms", ctypes.c_double),
                ("h2d_ms", ctypes.c_double), ("decode_ms", ctypes.c_double), ("index_ms", ctypes.c_double),
                ("ix_polls", ctypes.c_int64), ("ix_unreported", ctypes.c_int64), ("ix_fallback_chunks", ctypes.c_int64),
                ("ix_stale_entries", ctypes.c_int64)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


_LIB = None
TIMER_SLOTS = 25  # PQGPU_TIMER_SLOTS
ABI_VERSION = 8  # PQGPU_ABI_VERSION in include/pqgpu.h (struct layouts above)
_EXPORTS = [
    "pqgpu_abi_version", "pqgpu_status_string", "pqgpu_ctx_create", "pqgpu_ctx_destroy", "pqgpu_file_open",
    "pqgpu_file_close", "pqgpu_file_num_row_groups", "pqgpu_file_num_columns", "pqgpu_file_row_group_num_rows",
    "pqgpu_file_column", "pqgpu_file_chunk_meta", "pqgpu_batch_create", "pqgpu_batch_destroy", "pqgpu_batch_reset",
    "pqgpu_batch_add_chunk", "pqgpu_batch_add_file_chunk", "pqgpu_batch_upload", "pqgpu_batch_decode",
    "pqgpu_batch_sync", "pqgpu_batch_wait", "pqgpu_batch_num_chunks", "pqgpu_batch_chunk_status", "pqgpu_batch_chunk_result",
    "pqgpu_batch_copy_chunk", "pqgpu_batch_stats_get", "pqgpu_batch_kernel_timing", "pqgpu_batch_kernel_time",
    "pqgpu_batch_debug_counters", "pqgpu_batch_kernel_slot", "pqgpu_batch_chunk_pages", "pqgpu_batch_kernel_bytes",
    "pqgpu_copy", "pqgpu_pipeline_create", "pqgpu_pipeline_next", "pqgpu_pipeline_release", "pqgpu_pipeline_stats_get",
    "pqgpu_pipeline_destroy", "pqgpu_batch_copy_nested", "pqgpu_page_index_build", "pqgpu_page_index_chunk",
    "pqgpu_page_index_page", "pqgpu_page_index_walk_ms", "pqgpu_page_index_stats", "pqgpu_page_index_destroy", "pqgpu_parse_page_header",
    "pqgpu_batch_add_indexed_chunk", "pqgpu_batch_add_indexed_file_chunk", "pqgpu_dev_alloc", "pqgpu_dev_free",
    "pqgpu_batch_copy_group", "pqgpu_batch_share_ancestors",
]


def lib():
    """Load libpqgpu.so (raises if it was not built: there is no fallback)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"libpqgpu.so not built at {LIB_PATH}: run `make -C {_PKG}` (hipcc, gfx950)")
    L = ctypes.CDLL(LIB_PATH)
    P, E = ctypes.c_void_p, ctypes.POINTER(Error)
    sig = {
        "pqgpu_abi_version": ([], ctypes.c_int),
        "pqgpu_status_string": ([ctypes.c_int], ctypes.c_char_p),
        "pqgpu_ctx_create": ([ctypes.c_int, ctypes.POINTER(P), E], ctypes.c_int),
        "pqgpu_ctx_destroy": ([P], None),
        "pqgpu_file_open": ([P, ctypes.c_size_t, ctypes.POINTER(P), E], ctypes.c_int),
        "pqgpu_file_close": ([P], None),
        "pqgpu_file_num_row_groups": ([P], ctypes.c_int),
        "pqgpu_file_num_columns": ([P], ctypes.c_int),
        "pqgpu_file_row_group_num_rows": ([P, ctypes.c_int], ctypes.c_int64),
        "pqgpu_file_column": ([P, ctypes.c_int, ctypes.POINTER(ColumnInfo)], ctypes.c_int),
        "pqgpu_file_chunk_meta": ([P, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ChunkMeta), E], ctypes.c_int),
        "pqgpu_batch_create": ([P, ctypes.POINTER(P), E], ctypes.c_int),
        "pqgpu_batch_destroy": ([P], None),
        "pqgpu_batch_reset": ([P], ctypes.c_int),
        "pqgpu_batch_add_chunk": ([P, P, ctypes.c_size_t, ctypes.POINTER(ColumnInfo), ctypes.POINTER(ChunkMeta),
                                   ctypes.c_int, ctypes.POINTER(ctypes.c_int32), E], ctypes.c_int),
        "pqgpu_batch_add_file_chunk": ([P, P, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                        ctypes.POINTER(ctypes.c_int32), E], ctypes.c_int),
        "pqgpu_batch_upload": ([P, P, E], ctypes.c_int),
        "pqgpu_batch_decode": ([P, P, E], ctypes.c_int),
        "pqgpu_batch_sync": ([P, P, E], ctypes.c_int),
        "pqgpu_batch_wait": ([P, P, E], ctypes.c_int),
        "pqgpu_batch_num_chunks": ([P], ctypes.c_int),
        "pqgpu_batch_chunk_status": ([P, ctypes.c_int32, E], ctypes.c_int),
        "pqgpu_batch_chunk_result": ([P, ctypes.c_int32, ctypes.POINTER(ChunkResult), E], ctypes.c_int),
        "pqgpu_batch_copy_chunk": ([P, ctypes.c_int32, P, P, P, P, P, P, P, E], ctypes.c_int),
        "pqgpu_batch_stats_get": ([P, ctypes.POINTER(BatchStats)], ctypes.c_int),
        "pqgpu_batch_kernel_timing": ([P, ctypes.c_int], ctypes.c_int),
        "pqgpu_batch_debug_counters": ([P, P, ctypes.c_int], ctypes.c_int),
        "pqgpu_batch_kernel_time": ([P, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int64),
                                     ctypes.c_char_p, ctypes.c_size_t], ctypes.c_int),
        "pqgpu_batch_kernel_slot": ([P, ctypes.c_int, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int64),
                                     ctypes.c_char_p, ctypes.c_size_t], ctypes.c_int),
        "pqgpu_batch_chunk_pages": ([P, ctypes.c_int32, ctypes.POINTER(ctypes.c_int32), P, P, P, P, ctypes.c_int32, E],
                                    ctypes.c_int),
        "pqgpu_batch_kernel_bytes": ([P, ctypes.c_int, ctypes.POINTER(ctypes.c_int64)], ctypes.c_int),
        "pqgpu_copy": ([P, P, P, ctypes.c_size_t, E], ctypes.c_int),
        "pqgpu_batch_copy_nested": ([P, ctypes.c_int32, ctypes.c_int32, P, P, P, E], ctypes.c_int),
        "pqgpu_batch_copy_group": ([P, ctypes.c_int32, ctypes.c_int32, P, E], ctypes.c_int),
        "pqgpu_batch_share_ancestors": ([P, ctypes.c_int32, ctypes.c_int32, ctypes.POINTER(ctypes.c_int32), E], ctypes.c_int),
        "pqgpu_pipeline_create": ([P, P, P, ctypes.c_int32, P, ctypes.c_int32, ctypes.POINTER(PipelineOpts),
                                   ctypes.POINTER(P), E], ctypes.c_int),
        "pqgpu_pipeline_next": ([P, ctypes.POINTER(P), ctypes.POINTER(ctypes.c_int32), E], ctypes.c_int),
        "pqgpu_pipeline_release": ([P, P], ctypes.c_int),
        "pqgpu_pipeline_stats_get": ([P, ctypes.POINTER(PipelineStats)], ctypes.c_int),
        "pqgpu_pipeline_destroy": ([P], None),
        "pqgpu_page_index_build": ([P, P, ctypes.c_int64, ctypes.c_int64, ctypes.POINTER(ChunkMeta), ctypes.c_int32,
                                    ctypes.c_int32, P, ctypes.POINTER(P), E], ctypes.c_int),
        "pqgpu_page_index_chunk": ([P, ctypes.c_int32, ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int32)],
                                   ctypes.c_int),
        "pqgpu_page_index_page": ([P, ctypes.c_int32, ctypes.c_int32, ctypes.POINTER(PageHeader)], ctypes.c_int),
        "pqgpu_page_index_walk_ms": ([P], ctypes.c_double),
        "pqgpu_page_index_stats": ([P] + [ctypes.POINTER(ctypes.c_int32)] * 5, ctypes.c_int),
        "pqgpu_page_index_destroy": ([P], None),
        "pqgpu_parse_page_header": ([P, ctypes.c_size_t, ctypes.POINTER(PageHeader), ctypes.POINTER(ctypes.c_int64)],
                                    ctypes.c_int),
        "pqgpu_batch_add_indexed_chunk": ([P, P, ctypes.c_int32, P, ctypes.c_size_t, ctypes.POINTER(ColumnInfo),
                                           ctypes.c_int, ctypes.POINTER(ctypes.c_int32), E], ctypes.c_int),
        "pqgpu_batch_add_indexed_file_chunk": ([P, P, ctypes.c_int32, P, ctypes.c_int, ctypes.c_int,
                                                ctypes.POINTER(ctypes.c_int32), E], ctypes.c_int),
        "pqgpu_dev_alloc": ([P, ctypes.c_size_t, ctypes.POINTER(P), E], ctypes.c_int),
        "pqgpu_dev_free": ([P, P], None),
    }
    for name, (args, res) in sig.items():
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = res
    if L.pqgpu_abi_version() != ABI_VERSION:
        raise RuntimeError(f"{LIB_PATH}: ABI version {L.pqgpu_abi_version()}, these bindings need {ABI_VERSION}: rebuild it")
    _LIB = L
    return L


class DecodeError(Exception):
    """A reader error with the reference's error class (see ERROR_NAMES)."""

    def __init__(self, err):
        self.code = int(err.code)
        self.chunk = int(err.chunk)
        self.page = int(err.page)
        self.msg = err.msg.decode(errors="replace")
        super().__init__(f"[{ERROR_NAMES.get(self.code, self.code)}] chunk {self.chunk} page {self.page}: {self.msg}")


# Live handles, released in order (batches, then contexts) before the interpreter tears down
# modules: a batch left alive by an exception traceback would otherwise be destroyed by GC
# after its context or after the HIP runtime has shut down.
_live_batches = weakref.WeakSet()
_live_contexts = weakref.WeakSet()
_live_pipelines = weakref.WeakSet()  # closed first: they own batches, streams and a page-locked file
_live_indexes = weakref.WeakSet()    # page indexes and the device copies of file bytes they keep


@atexit.register
def _release_all():
    for p in list(_live_pipelines):
        p.close()
    for x in list(_live_indexes):
        x.close()
    for b in list(_live_batches):
        b.close()
    for c in list(_live_contexts):
        c.close()


def _check(rc, err):
    if rc:
        raise DecodeError(err)


class Context:
    """One MI355X device (pqgpu_ctx). HIP device visibility follows HIP_VISIBLE_DEVICES."""

    def __init__(self, device=0):
        self._h = ctypes.c_void_p()
        err = Error()
        _check(lib().pqgpu_ctx_create(device, ctypes.byref(self._h), ctypes.byref(err)), err)
        self.device = device
        _live_contexts.add(self)

    def close(self):
        if self._h:
            lib().pqgpu_ctx_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class File:
    """Parsed footer + schema (ReadFileMetaData + makeSchema). Keeps `data` alive."""

    def __init__(self, data):
        self.data = bytes(data)
        self._buf = ctypes.create_string_buffer(self.data, len(self.data))
        self._h = ctypes.c_void_p()
        err = Error()
        _check(lib().pqgpu_file_open(ctypes.addressof(self._buf), len(self.data), ctypes.byref(self._h),
                                     ctypes.byref(err)), err)

    def close(self):
        if self._h:
            lib().pqgpu_file_close(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def num_row_groups(self):
        return lib().pqgpu_file_num_row_groups(self._h)

    @property
    def num_columns(self):
        return lib().pqgpu_file_num_columns(self._h)

    def row_group_num_rows(self, rg):
        return lib().pqgpu_file_row_group_num_rows(self._h, rg)

    def column(self, col):
        ci = ColumnInfo()
        if lib().pqgpu_file_column(self._h, col, ctypes.byref(ci)):
            raise IndexError(col)
        return ci

    def chunk_meta(self, rg, col):
        m, err = ChunkMeta(), Error()
        _check(lib().pqgpu_file_chunk_meta(self._h, rg, col, ctypes.byref(m), ctypes.byref(err)), err)
        return m

    def column_paths(self):
        return [self.column(i).path.decode() for i in range(self.num_columns)]


class ColumnData:
    """One decoded column chunk, in the reference's terms plus Arrow-style extras."""

    def __init__(self, info, res, values, offsets, payload, dlev, rlev, validity, lists):
        self.path = info.path.decode()
        self.physical_type = info.physical_type
        self.max_def, self.max_rep = info.max_def, info.max_rep
        self.num_slots, self.num_values, self.num_records = res.num_slots, res.num_values, res.num_records
        self.values_raw = values     # fixed width: ndarray (INT96: (n,12) uint8)
        self.offsets = offsets       # BYTE_ARRAY: int32[n+1]
        self.payload = payload       # BYTE_ARRAY: bytes
        self.validity = validity     # uint32 words or None
        self.list_offsets = lists    # int32[records+1] or None
        n = self.num_slots
        if dlev is not None:
            self.dLevels = dlev.astype(np.int32)
        elif self.max_def == 1:      # validity bits ARE the def levels when maxD == 1
            self.dLevels = self.validity_bits().astype(np.int32)
        else:
            self.dLevels = np.zeros(n, np.int32)
        self.rLevels = rlev.astype(np.int32) if rlev is not None else np.zeros(n, np.int32)

    def validity_bits(self):
        if self.validity is None:
            return np.ones(self.num_slots, np.uint8)
        b = np.unpackbits(self.validity.view(np.uint8), bitorder="little")
        return b[: self.num_slots]

    @property
    def values(self):
        """Non-null values in order; byte arrays as a list of bytes."""
        if self.offsets is not None:
            o = self.offsets
            return [self.payload[o[i]:o[i + 1]] for i in range(self.num_values)]
        return self.values_raw


class Batch:
    """pqgpu_batch: chunks decoded together with one set of kernel launches."""

    def __init__(self, ctx):
        self.ctx = ctx
        self._h = ctypes.c_void_p()
        err = Error()
        _check(lib().pqgpu_batch_create(ctx._h if ctx is not None else None, ctypes.byref(self._h),
                                        ctypes.byref(err)), err)
        self._files = []
        self._infos = []
        _live_batches.add(self)

    def close(self):
        if self._h:
            lib().pqgpu_batch_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def reset(self):
        lib().pqgpu_batch_reset(self._h)
        self._files, self._infos = [], []

    def add_file_chunk(self, f, rg, col, validate_crc=False):
        """readRowGroupData for one (row group, column). Returns (chunk_id, error or None)."""
        cid = ctypes.c_int32(-1)
        err = Error()
        rc = lib().pqgpu_batch_add_file_chunk(self._h, f._h, rg, col, int(validate_crc), ctypes.byref(cid),
                                              ctypes.byref(err))
        self._files.append(f)
        self._infos.append(f.column(col))
        return cid.value, (DecodeError(err) if rc else None)

    def add_indexed_chunk(self, ix, k, f, col, validate_crc=False):
        """add_file_chunk for chunk k of a PageIndex (page headers and CRC verdicts from the device
        walk, UNCOMPRESSED page bodies gathered from the resident bytes at upload)."""
        cid = ctypes.c_int32(-1)
        err = Error()
        rc = lib().pqgpu_batch_add_indexed_file_chunk(self._h, ix._h, k, f._h, col, int(validate_crc),
                                                      ctypes.byref(cid), ctypes.byref(err))
        self._files.append(f)
        self._files.append(ix)  # upload gathers page bodies from the index's device buffer
        self._infos.append(f.column(col))
        return cid.value, (DecodeError(err) if rc else None)

    def upload(self):
        err = Error()
        _check(lib().pqgpu_batch_upload(self._h, None, ctypes.byref(err)), err)

    def decode(self):
        err = Error()
        _check(lib().pqgpu_batch_decode(self._h, None, ctypes.byref(err)), err)

    def sync(self):
        """Wait; returns the first error (DecodeError) or None."""
        err = Error()
        rc = lib().pqgpu_batch_sync(self._h, None, ctypes.byref(err))
        return DecodeError(err) if rc else None

    def wait(self):
        """Wait for the queued decodes on the device (no error collection: sync() does that)."""
        err = Error()
        _check(lib().pqgpu_batch_wait(self._h, None, ctypes.byref(err)), err)

    def status(self, cid):
        err = Error()
        rc = lib().pqgpu_batch_chunk_status(self._h, cid, ctypes.byref(err))
        return DecodeError(err) if rc else None

    def stats(self):
        s = BatchStats()
        lib().pqgpu_batch_stats_get(self._h, ctypes.byref(s))
        return s

    def debug_counters(self, reset=True):
        out = np.zeros(64, np.uint64)
        lib().pqgpu_batch_debug_counters(self._h, out.ctypes.data_as(ctypes.c_void_p), int(reset))
        return out

    def kernel_timing(self, enable=True):
        lib().pqgpu_batch_kernel_timing(self._h, int(enable))

    def kernel_time(self):
        ms, n = ctypes.c_double(), ctypes.c_int64()
        name = ctypes.create_string_buffer(64)
        lib().pqgpu_batch_kernel_time(self._h, ctypes.byref(ms), ctypes.byref(n), name, 64)
        return ms.value, n.value, name.value.decode()

    def kernel_times(self):
        """{kernel name: (average ms per launch, launches, algorithmic bytes per launch)} for every
        timed launch slot that ran."""
        out = {}
        for k in range(TIMER_SLOTS):
            ms, n, nb = ctypes.c_double(), ctypes.c_int64(), ctypes.c_int64()
            name = ctypes.create_string_buffer(64)
            lib().pqgpu_batch_kernel_slot(self._h, k, ctypes.byref(ms), ctypes.byref(n), name, 64)
            lib().pqgpu_batch_kernel_bytes(self._h, k, ctypes.byref(nb))
            if n.value:
                out[name.value.decode()] = (ms.value, n.value, nb.value)
        return out

    def pages(self, cid):
        """Per-page split of chunk `cid` (pageReader granularity): array of
        (slot_first, slot_count, value_first, value_count) rows."""
        err = Error()
        n = ctypes.c_int32()
        _check(lib().pqgpu_batch_chunk_pages(self._h, cid, ctypes.byref(n), None, None, None, None, 0,
                                             ctypes.byref(err)), err)
        out = np.zeros((4, n.value), np.int64)
        ptr = [out[k].ctypes.data_as(ctypes.c_void_p) for k in range(4)]
        _check(lib().pqgpu_batch_chunk_pages(self._h, cid, ctypes.byref(n), *ptr, n.value, ctypes.byref(err)), err)
        return out.T.copy()

    def result(self, cid, copy=True, partial=False):
        """ColumnData for chunk `cid` (raises DecodeError if that chunk failed). partial=True returns
        (ColumnData of the pages decoded before a failing page, or None; DecodeError or None): the
        rows the reference's lazy page reader returns before the page that fails
        (data_store.go:236-260)."""
        err = Error()
        r = ChunkResult()
        rc = lib().pqgpu_batch_chunk_result(self._h, cid, ctypes.byref(r), ctypes.byref(err))
        if partial:
            e = DecodeError(err) if rc else None
            if rc and not r.num_slots:
                return None, e
            data = self._copy(cid, r, err) if copy else r
            return data, e
        _check(rc, err)
        if not copy:
            return r
        return self._copy(cid, r, err)

    def _copy(self, cid, r, err):
        info = self._infos[cid]
        ns, nv = r.num_slots, r.num_values
        t = r.physical_type
        vals = offs = pay = dl = rl = valid = lists = None
        if r.value_width:
            if t == INT96 or (t == FIXED_LEN_BYTE_ARRAY):
                vals = np.zeros((nv, r.value_width), np.uint8)
            else:
                vals = np.zeros(nv, _DTYPES[t])
        else:
            offs = np.zeros(nv + 1, np.int32)
            pay = np.zeros(max(r.payload_bytes, 1), np.uint8)
        if r.def_levels:
            dl = np.zeros(ns, np.uint8)
        if r.rep_levels:
            rl = np.zeros(ns, np.uint8)
        if r.validity:
            valid = np.zeros((ns + 31) // 32, np.uint32)
        if r.list_offsets:
            lists = np.zeros(r.num_records + 1, np.int32)

        def ptr(a):
            return None if a is None else a.ctypes.data_as(ctypes.c_void_p)

        rc = lib().pqgpu_batch_copy_chunk(self._h, cid, ptr(vals), ptr(offs), ptr(pay), ptr(dl), ptr(rl),
                                          ptr(valid), ptr(lists), ctypes.byref(err))
        if rc and not r.num_slots:
            _check(rc, err)
        payload = pay[: r.payload_bytes].tobytes() if pay is not None else None
        cd = ColumnData(info, r, vals, offs, payload, dl, rl, valid, lists)
        cd.nested = []  # Arrow-style list levels, outermost first: (offsets int32[n+1], validity bits uint8[n])
        cd.element_validity = None
        for k in range(r.nest_levels):
            n = r.num_lists[k]
            lo = np.zeros(n + 1, np.int32)
            lv = np.zeros(max((n + 31) // 32, 1), np.uint32)
            ev = np.zeros(max((r.num_elements + 31) // 32, 1), np.uint32) if k == 0 else None
            _check(lib().pqgpu_batch_copy_nested(self._h, cid, k, lo.ctypes.data_as(ctypes.c_void_p),
                                                 lv.ctypes.data_as(ctypes.c_void_p),
                                                 None if ev is None else ev.ctypes.data_as(ctypes.c_void_p),
                                                 ctypes.byref(err)), err)
            cd.nested.append((lo, np.unpackbits(lv.view(np.uint8), bitorder="little")[:n]))
            if ev is not None:
                cd.element_validity = np.unpackbits(ev.view(np.uint8), bitorder="little")[: r.num_elements]
        # struct validity of the OPTIONAL groups on the path: [(dotted group path, validity bits uint8[n])]
        cd.groups = []
        parts = info.path.decode().split(".")
        for g in range(r.num_groups):
            n = r.group_entries[g]
            gv = np.zeros(max((n + 31) // 32, 1), np.uint32)
            _check(lib().pqgpu_batch_copy_group(self._h, cid, g, gv.ctypes.data_as(ctypes.c_void_p), ctypes.byref(err)), err)
            cd.groups.append((".".join(parts[: info.group_node[g] + 1]),
                              np.unpackbits(gv.view(np.uint8), bitorder="little")[:n]))
        return cd

    def share_ancestors(self, cid_a, cid_b):
        """pqgpu_batch_share_ancestors: True when the two leaves' common ancestors (list levels and
        OPTIONAL groups on the shared path prefix) decoded identically; chunk b's result then carries
        chunk a's arrays for them (one shared offsets array per list level)."""
        eq, err = ctypes.c_int32(0), Error()
        _check(lib().pqgpu_batch_share_ancestors(self._h, cid_a, cid_b, ctypes.byref(eq), ctypes.byref(err)), err)
        return bool(eq.value)


class _PipelineBatch(Batch):
    """A batch owned by a Pipeline (valid until the pipeline moves past it)."""

    def __init__(self, handle, infos):
        self.ctx = None
        self._h = handle
        self._files = []
        self._infos = infos

    def close(self):
        self._h = ctypes.c_void_p()


class Pipeline:
    """pqgpu_pipeline: row groups of `f` streamed through `depth` batches (host planning and H2D
    of later row groups overlap the decode of earlier ones). Iterating yields
    (row_group, batch, error or None) in row-group order; a yielded batch is released when the
    iteration moves on. Chunk ids in a batch follow `cols`."""

    def __init__(self, ctx, f, row_groups=None, cols=None, depth=3, threads=0, validate_crc=False,
                 device_index=False):
        self.ctx, self.f = ctx, f
        self.cols = list(range(f.num_columns)) if cols is None else list(cols)
        self._infos = [f.column(c) for c in self.cols]
        rgs = None if row_groups is None else (ctypes.c_int32 * len(row_groups))(*row_groups)
        cs = (ctypes.c_int32 * len(self.cols))(*self.cols)
        opts = PipelineOpts(depth, threads, int(validate_crc), int(device_index))
        self._h = ctypes.c_void_p()
        err = Error()
        _check(lib().pqgpu_pipeline_create(ctx._h, f._h, rgs, len(row_groups) if row_groups is not None else 0, cs,
                                           len(self.cols), ctypes.byref(opts), ctypes.byref(self._h),
                                           ctypes.byref(err)), err)
        self._out = None
        _live_pipelines.add(self)

    def __iter__(self):
        while True:
            self._release()
            b, rg, err = ctypes.c_void_p(), ctypes.c_int32(), Error()
            rc = lib().pqgpu_pipeline_next(self._h, ctypes.byref(b), ctypes.byref(rg), ctypes.byref(err))
            if not b.value:
                _check(rc, err)
                return
            self._out = _PipelineBatch(b, self._infos)
            yield rg.value, self._out, (DecodeError(err) if rc else None)

    def _release(self):
        if self._out is not None:
            lib().pqgpu_pipeline_release(self._h, self._out._h)
            self._out.close()
            self._out = None

    def stats(self):
        s = PipelineStats()
        lib().pqgpu_pipeline_stats_get(self._h, ctypes.byref(s))
        return s.as_dict()

    def close(self):
        if self._h:
            self._release()
            lib().pqgpu_pipeline_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class DeviceBuffer:
    """Device memory on libpqgpu's runtime holding `data` (pqgpu_dev_alloc + pqgpu_copy)."""

    def __init__(self, ctx, data=None, pad=64, src_addr=None, size=None):
        """`data` (bytes-like), or `size` bytes at host address `src_addr` (no intermediate copy)."""
        self.ctx, self.size = ctx, (len(data) if src_addr is None else size)
        self.ptr = ctypes.c_void_p()
        _live_indexes.add(self)
        err = Error()
        _check(lib().pqgpu_dev_alloc(ctx._h, self.size + pad, ctypes.byref(self.ptr), ctypes.byref(err)), err)
        if self.size:
            if src_addr is None:
                src = ctypes.create_string_buffer(bytes(data), self.size)
                src_addr = ctypes.addressof(src)
            copy(ctx, self.ptr.value, src_addr, self.size)

    def close(self):
        if self.ptr and self.ptr.value:
            lib().pqgpu_dev_free(self.ctx._h, self.ptr)
            self.ptr = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def parse_page_header(buf):
    """The host's PageHeader decode: (PageHeader, consumed) or (None, consumed) on a Thrift error."""
    h, n = PageHeader(), ctypes.c_int64()
    src = ctypes.create_string_buffer(bytes(buf), len(buf))
    rc = lib().pqgpu_parse_page_header(ctypes.addressof(src), len(buf), ctypes.byref(h), ctypes.byref(n))
    return (None if rc else h), n.value


class PageIndex:
    """pqgpu_page_index: the page headers of column chunks walked on the GPU over resident file bytes
    (readPages' header loop, chunk_reader.go:182-263, and readPageBlock's CRC32 check, :173-177)."""

    def __init__(self, ctx, dev_ptr, file_offset, length, metas, validate_crc=False, keep=None):
        self.ctx, self._keep = ctx, keep
        self.metas = list(metas)
        arr = (ChunkMeta * max(len(self.metas), 1))(*self.metas)
        self._h = ctypes.c_void_p()
        err = Error()
        _check(lib().pqgpu_page_index_build(ctx._h, ctypes.c_void_p(dev_ptr), file_offset, length, arr,
                                            len(self.metas), int(validate_crc), None, ctypes.byref(self._h),
                                            ctypes.byref(err)), err)
        _live_indexes.add(self)

    @classmethod
    def for_chunks(cls, ctx, f, chunks, validate_crc=False, whole_file=False):
        """Index the (row group, column) chunks of File f: their byte range (or the whole file) is
        copied to the device once."""
        metas = [f.chunk_meta(rg, c) for rg, c in chunks]
        if whole_file or not metas:
            lo, hi = 0, len(f.data)
        else:
            st = [m.dictionary_page_offset if m.dictionary_page_offset >= 0 else m.data_page_offset for m in metas]
            lo = max(0, min(st))
            hi = min(len(f.data), max(s + max(m.total_compressed_size, 0) for s, m in zip(st, metas)))
            hi = max(hi, lo)
        buf = DeviceBuffer(ctx, src_addr=ctypes.addressof(f._buf) + lo, size=hi - lo)
        return cls(ctx, buf.ptr.value, lo, hi - lo, metas, validate_crc, keep=buf)

    def chunk(self, k):
        n, st = ctypes.c_int32(), ctypes.c_int32()
        if lib().pqgpu_page_index_chunk(self._h, k, ctypes.byref(n), ctypes.byref(st)):
            raise IndexError(k)
        return n.value, st.value

    def page(self, k, i):
        h = PageHeader()
        if lib().pqgpu_page_index_page(self._h, k, i, ctypes.byref(h)):
            raise IndexError((k, i))
        return h

    @property
    def walk_ms(self):
        return lib().pqgpu_page_index_walk_ms(self._h)

    def stats(self):
        """{polls, unreported, fallback_chunks, overflowed, stale_entries} of the build (pqgpu_page_index_stats)."""
        v = [ctypes.c_int32() for _ in range(5)]
        lib().pqgpu_page_index_stats(self._h, *[ctypes.byref(x) for x in v])
        return dict(zip(("polls", "unreported", "fallback_chunks", "overflowed", "stale_entries"), (x.value for x in v)))

    def close(self):
        if self._h:
            lib().pqgpu_page_index_destroy(self._h)
            self._h = ctypes.c_void_p()
        if self._keep is not None:
            self._keep.close()
            self._keep = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def copy(ctx, dst, src, nbytes):
    """pqgpu_copy: hipMemcpy(hipMemcpyDefault) on the library's HIP runtime (integer addresses)."""
    err = Error()
    _check(lib().pqgpu_copy(ctx._h, ctypes.c_void_p(dst), ctypes.c_void_p(src), nbytes, ctypes.byref(err)), err)


class FileReader:
    """Mirror of goparquet.FileReader for the decode path (file_reader.go)."""

    def __init__(self, data, *columns, ctx=None, validate_crc=False):
        self.file = File(data)
        self.ctx = ctx or Context(0)
        self.validate_crc = validate_crc
        paths = self.file.column_paths()
        self.selected = [i for i, p in enumerate(paths) if not columns or p in columns or p.split(".")[0] in columns]
        self.rowGroupPosition = 0

    def NumRowGroups(self):
        return self.file.num_row_groups

    def NumRows(self):
        return sum(self.file.row_group_num_rows(i) for i in range(self.file.num_row_groups))

    def ReadRowGroupData(self, rg):
        """readRowGroupData (chunk_reader.go:375-404): decode every selected column chunk of row group rg.
        Returns {path: ColumnData}; raises DecodeError with the first error in column order."""
        b = Batch(self.ctx)
        try:
            ids = []
            for c in self.selected:
                cid, e = b.add_file_chunk(self.file, rg, c, self.validate_crc)
                if e is not None:
                    raise e
                ids.append((c, cid))
            b.decode()
            e = b.sync()
            if e is not None:
                raise e
            return {self.file.column(c).path.decode(): b.result(cid) for c, cid in ids}
        finally:
            b.close()


def NewFileReader(data, *columns, **kw):
    return FileReader(data, *columns, **kw)
