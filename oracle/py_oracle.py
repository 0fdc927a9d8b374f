"""ctypes binding for the CPU oracle (oracle/liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg as the parity checker. The product path
(parquet-go-1_amd/) never imports this module.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

# parquet.Type -> numpy dtype of one decoded value (byte arrays: None)
TYPE_DTYPES = {0: np.uint8, 1: np.int32, 2: np.int64, 3: None, 4: np.uint32, 5: np.uint64, 6: None, 7: None}


class ColumnInfo(ctypes.Structure):
    _fields_ = [("physical_type", ctypes.c_int32), ("type_length", ctypes.c_int32),
                ("max_def", ctypes.c_int32), ("max_rep", ctypes.c_int32),
                ("repetition", ctypes.c_int32), ("path", ctypes.c_char * 256),
                ("path_len", ctypes.c_int32), ("node_rep", ctypes.c_int32 * 64)]


class ChunkResult(ctypes.Structure):
    _fields_ = [("err_code", ctypes.c_int32), ("err_page", ctypes.c_int32),
                ("err_msg", ctypes.c_char * 256), ("num_slots", ctypes.c_int64),
                ("num_values", ctypes.c_int64), ("value_width", ctypes.c_int32),
                ("num_pages", ctypes.c_int32),
                ("def_levels", ctypes.POINTER(ctypes.c_int32)),
                ("rep_levels", ctypes.POINTER(ctypes.c_int32)),
                ("values", ctypes.POINTER(ctypes.c_uint8)), ("values_bytes", ctypes.c_int64),
                ("offsets", ctypes.POINTER(ctypes.c_int64))]


def build():
    """Compile liboracle.so (gcc, zlib)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _LIB
    if _LIB is None:
        path = os.environ.get("PQ_ORACLE_LIB") or os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            build()
        L = ctypes.CDLL(path)
        L.or_file_open.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_void_p),
                                   ctypes.c_char_p, ctypes.c_size_t]
        L.or_file_close.argtypes = [ctypes.c_void_p]
        L.or_file_num_row_groups.argtypes = [ctypes.c_void_p]
        L.or_file_num_columns.argtypes = [ctypes.c_void_p]
        L.or_file_row_group_num_rows.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.or_file_row_group_num_rows.restype = ctypes.c_int64
        L.or_file_column_info.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ColumnInfo)]
        L.or_read_chunk.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                    ctypes.POINTER(ChunkResult)]
        L.or_chunk_result_free.argtypes = [ctypes.POINTER(ChunkResult)]
        L.or_hybrid_decode.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int64,
                                       ctypes.c_void_p, ctypes.POINTER(ctypes.c_int64)]
        L.or_delta_decode64.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int64, ctypes.c_void_p,
                                        ctypes.POINTER(ctypes.c_int64)]
        L.or_delta_decode32.argtypes = L.or_delta_decode64.argtypes
        L.or_unpack8_int32.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
        L.or_unpack8_int64.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
        _LIB = L
    return _LIB


class OracleError(Exception):
    def __init__(self, code, page, msg):
        super().__init__(f"oracle error {code} page {page}: {msg}")
        self.code, self.page, self.msg = code, page, msg


class ChunkData:
    """Decoded column chunk: the reference's (values, dLevels, rLevels) per page, concatenated."""

    def __init__(self, def_levels, rep_levels, values, offsets, num_values, physical_type, num_pages):
        self.def_levels = def_levels
        self.rep_levels = rep_levels
        self.values = values          # fixed width: ndarray; byte arrays: bytes payload
        self.offsets = offsets        # byte arrays: int64 ndarray (num_values+1), else None
        self.num_values = num_values
        self.physical_type = physical_type
        self.num_pages = num_pages


class File:
    def __init__(self, data: bytes):
        self._buf = ctypes.create_string_buffer(bytes(data), len(data))
        self._h = ctypes.c_void_p()
        err = ctypes.create_string_buffer(256)
        rc = lib().or_file_open(ctypes.addressof(self._buf), len(data), ctypes.byref(self._h), err, 256)
        if rc:
            raise OracleError(rc, -1, err.value.decode(errors="replace"))

    def close(self):
        if self._h:
            lib().or_file_close(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def num_row_groups(self):
        return lib().or_file_num_row_groups(self._h)

    @property
    def num_columns(self):
        return lib().or_file_num_columns(self._h)

    def row_group_num_rows(self, rg):
        return lib().or_file_row_group_num_rows(self._h, rg)

    def column_info(self, col):
        ci = ColumnInfo()
        if lib().or_file_column_info(self._h, col, ctypes.byref(ci)):
            raise IndexError(col)
        return ci

    def read_chunk(self, rg, col, validate_crc=False):
        r = ChunkResult()
        rc = lib().or_read_chunk(self._h, rg, col, int(validate_crc), ctypes.byref(r))
        ci = self.column_info(col)
        try:
            if rc:
                raise OracleError(rc, r.err_page, r.err_msg.decode(errors="replace"))
            ns, nv = r.num_slots, r.num_values
            dl = np.ctypeslib.as_array(r.def_levels, (ns,)).copy() if ns else np.zeros(0, np.int32)
            rl = np.ctypeslib.as_array(r.rep_levels, (ns,)).copy() if ns else np.zeros(0, np.int32)
            raw = ctypes.string_at(r.values, r.values_bytes) if r.values_bytes else b""
            offs = None
            if r.value_width == 0:
                offs = np.ctypeslib.as_array(r.offsets, (nv + 1,)).copy() if r.offsets else np.zeros(1, np.int64)
                vals = raw
            elif ci.physical_type == 3:
                vals = np.frombuffer(raw, np.uint8).reshape(-1, 12).copy()
            else:
                vals = np.frombuffer(raw, TYPE_DTYPES[ci.physical_type]).copy()
            return ChunkData(dl, rl, vals, offs, nv, ci.physical_type, r.num_pages)
        finally:
            lib().or_chunk_result_free(ctypes.byref(r))


def unpack8_int32(data: bytes, bw: int):
    out = (ctypes.c_int32 * 8)()
    buf = ctypes.create_string_buffer(bytes(data) + b"\0" * 8)
    lib().or_unpack8_int32(buf, bw, out)
    return list(out)


def unpack8_int64(data: bytes, bw: int):
    out = (ctypes.c_int64 * 8)()
    buf = ctypes.create_string_buffer(bytes(data) + b"\0" * 8)
    lib().or_unpack8_int64(buf, bw, out)
    return list(out)


def hybrid_decode(data: bytes, bw: int, n: int):
    out = np.zeros(n, np.int32)
    dec = ctypes.c_int64()
    buf = ctypes.create_string_buffer(bytes(data), max(1, len(data)))
    rc = lib().or_hybrid_decode(buf, len(data), bw, n, out.ctypes.data, ctypes.byref(dec))
    return rc, out[: dec.value]


def delta_decode(data: bytes, n: int, bits=64):
    out = np.zeros(n, np.int64 if bits == 64 else np.int32)
    dec = ctypes.c_int64()
    buf = ctypes.create_string_buffer(bytes(data), max(1, len(data)))
    fn = lib().or_delta_decode64 if bits == 64 else lib().or_delta_decode32
    rc = fn(buf, len(data), n, out.ctypes.data, ctypes.byref(dec))
    return rc, out[: dec.value]
