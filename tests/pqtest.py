"""Shared helpers for the parity tests: fixture discovery, oracle decoding,
pyarrow-derived expectations, and bit-exact comparison of GPU output with
the oracle (CPU restatement of the reference, oracle/)."""
import glob
import io
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

# Fixtures whose every chunk must decode without error (values compared with pyarrow too).
VALID = ["cfg1", "cfg2_v2_small", "cfg3_small", "cfg4_small", "cfg5_small", "types_v1", "types_v2", "types_dict",
         "edge_nulls_v1", "edge_nulls_v2", "edge_tiny_pages", "edge_delta32", "edge_delta64_wide",
         "cfg2_snappy_v1", "cfg4_v2", "edge_empty", "dlba_v1", "dba_v2", "dba_v1_snappy", "cfg1_full",
         "cfg3_dict64k", "crc_v1", "crc_v1_flipped"]
# Fixtures with a known reference error: name -> (error class, data page index or -1 for chunk level).
EXPECTED_ERRORS = {
    "bad_dict_index": (5, 1),      # dict: invalid index (type_dict.go:52-54) on the 2nd data page
    "bad_delta_width": (3, 1),     # invalid miniblock bit width 40 in page 1 init() (deltabp_decoder.go:101-105)
    "bad_def_empty_run": (3, 2),   # "rle: empty RLE run" (hybrid_decoder.go:159-161) in def levels of page 2
    "edge_delta_q1": (1, 0),       # Q1 look-ahead: N = 257 needs a block header no writer emits -> io.EOF
    "cfg2_gzip_v2": (7, 1),        # Q5: V2 page written with is_compressed=false is gunzipped anyway (page_v2.go:125)
}
ALL = sorted(os.path.basename(p)[:-8] for p in glob.glob(os.path.join(GOLDEN, "*.parquet")))


def load(name):
    with open(os.path.join(GOLDEN, name + ".parquet"), "rb") as f:
        return f.read()


def oracle_decode(data):
    """[(rg, col, ChunkData | OracleError)] for every chunk, via the CPU oracle."""
    import py_oracle as O
    f = O.File(data)
    out = []
    for rg in range(f.num_row_groups):
        for col in range(f.num_columns):
            try:
                out.append((rg, col, f.read_chunk(rg, col)))
            except O.OracleError as e:
                out.append((rg, col, e))
    return out


def pyarrow_flat(data, col_name):
    """(non-null values as raw bits/bytes, validity) for a flat column, per row group."""
    import pyarrow as pa
    import pyarrow.parquet as pq
    pf = pq.ParquetFile(io.BytesIO(data))
    res = []
    for rg in range(pf.num_row_groups):
        arr = pf.read_row_group(rg, columns=[col_name]).column(0).combine_chunks()
        valid = ~np.asarray(arr.is_null()) if arr.null_count else np.ones(len(arr), bool)
        t = arr.type
        nn = arr.filter(pa.compute.invert(arr.is_null())) if arr.null_count else arr
        if pa.types.is_boolean(t):
            vals = np.asarray(nn.to_numpy(zero_copy_only=False), np.uint8)
        elif pa.types.is_timestamp(t):
            vals = None  # INT96: compared with the oracle only
        elif pa.types.is_binary(t) or pa.types.is_string(t) or pa.types.is_fixed_size_binary(t):
            vals = [bytes(x.as_py() if not isinstance(x.as_py(), str) else x.as_py().encode()) for x in nn]
        elif pa.types.is_floating(t):
            np_t = np.uint32 if t == pa.float32() else np.uint64
            vals = nn.to_numpy(zero_copy_only=False).view(np_t)
        else:
            vals = nn.to_numpy(zero_copy_only=False)
        res.append((vals, valid))
    return res


def oracle_values(cd):
    """Oracle ChunkData values as comparable python/numpy objects."""
    if cd.offsets is not None:
        o = cd.offsets
        return [cd.values[o[i]:o[i + 1]] for i in range(cd.num_values)]
    return cd.values


def assert_chunk_equal(gpu, orc, where=""):
    """Bit-exact comparison of a GPU ColumnData with an oracle ChunkData."""
    assert gpu.num_slots == len(orc.def_levels), f"{where}: slots {gpu.num_slots} != {len(orc.def_levels)}"
    assert gpu.num_values == orc.num_values, f"{where}: values {gpu.num_values} != {orc.num_values}"
    np.testing.assert_array_equal(gpu.dLevels, orc.def_levels, err_msg=f"{where}: def levels")
    np.testing.assert_array_equal(gpu.rLevels, orc.rep_levels, err_msg=f"{where}: rep levels")
    if gpu.max_def > 0:
        np.testing.assert_array_equal(gpu.validity_bits(), (orc.def_levels == gpu.max_def).astype(np.uint8),
                                      err_msg=f"{where}: validity")
    if orc.offsets is not None and gpu.offsets is None:
        # FIXED_LEN_BYTE_ARRAY: the oracle keeps the reference's []byte values, the GPU a fixed-width array
        g = np.asarray(gpu.values_raw)
        w = g.shape[1] if g.ndim == 2 else 0
        assert np.all(np.diff(orc.offsets) == w), f"{where}: FLBA lengths"
        assert g.tobytes() == orc.values, f"{where}: FLBA bytes differ"
    elif orc.offsets is not None:
        assert gpu.offsets is not None, where
        np.testing.assert_array_equal(gpu.offsets.astype(np.int64), orc.offsets, err_msg=f"{where}: offsets")
        assert gpu.payload == orc.values, f"{where}: payload differs"
    else:
        g = np.asarray(gpu.values_raw)
        o = np.asarray(orc.values)
        assert g.tobytes() == o.tobytes(), f"{where}: values differ (first diff at " \
            f"{int(np.argmax(g.reshape(len(g), -1).view(np.uint8) != o.reshape(len(o), -1).view(np.uint8)))})"
    if gpu.max_rep > 0:
        starts = np.flatnonzero(orc.rep_levels == 0)
        exp = np.append(starts, len(orc.rep_levels)).astype(np.int32)
        np.testing.assert_array_equal(gpu.list_offsets, exp, err_msg=f"{where}: list offsets")


def schema_levels(node_reps):
    """From the repetition types of the path's nodes (0 REQUIRED, 1 OPTIONAL, 2 REPEATED; the
    leaf last): [(null_def, def, node)] per REPEATED node, [(def, depth, node)] per OPTIONAL group,
    and maxD (schema.go:893-990: every non-REQUIRED node adds a definition level, every REPEATED
    one a repetition level)."""
    d = r = 0
    lists, groups = [], []
    for i, t in enumerate(node_reps):
        d0 = d
        if t != 0:
            d += 1
        if t == 2:
            r += 1
            lists.append((d0, d, i))
        elif t == 1 and i < len(node_reps) - 1:
            groups.append((d, r, i))
    return lists, groups, d
