"""CPU tests of the C-ABI library: it loads, exports every symbol declared in
include/pqgpu.h, parses footers/schemas like the oracle, and its host-side
page-header validation (readChunk/readPages) reports the same errors as the
oracle. No GPU compute is called here."""
import os
import re

import numpy as np
import pytest

import pqgpu
import pqtest
import py_oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared_symbols():
    src = open(os.path.join(ROOT, "include", "pqgpu.h")).read()
    return sorted(set(re.findall(r"\b(pqgpu_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_header_symbols():
    L = pqgpu.lib()
    syms = _declared_symbols()
    assert len(syms) >= 25
    for s in syms:
        assert hasattr(L, s), s
    assert set(pqgpu._EXPORTS) <= set(syms)
    assert L.pqgpu_abi_version() == pqgpu.ABI_VERSION == 8


def test_status_strings():
    L = pqgpu.lib()
    assert L.pqgpu_status_string(1) == b"EOF"
    assert L.pqgpu_status_string(5) == b"dict: invalid index"


@pytest.mark.parametrize("name", pqtest.ALL)
def test_file_metadata_matches_oracle(name):
    data = pqtest.load(name)
    try:
        of = O.File(data)
    except O.OracleError as e:
        with pytest.raises(pqgpu.DecodeError) as ei:
            pqgpu.File(data)
        assert ei.value.code == e.code
        return
    gf = pqgpu.File(data)
    assert gf.num_row_groups == of.num_row_groups
    assert gf.num_columns == of.num_columns
    for c in range(of.num_columns):
        a, b = gf.column(c), of.column_info(c)
        assert (a.physical_type, a.type_length, a.max_def, a.max_rep, a.path) == \
               (b.physical_type, b.type_length, b.max_def, b.max_rep, b.path)


def _plan_errors(data):
    """Host-side (readPages) errors of a plan-only batch, per chunk."""
    f = pqgpu.File(data)
    b = pqgpu.Batch(None)
    out = {}
    for rg in range(f.num_row_groups):
        for col in range(f.num_columns):
            cid, e = b.add_file_chunk(f, rg, col)
            out[(rg, col)] = e
    b.close()
    return out


@pytest.mark.parametrize("name", pqtest.ALL)
def test_host_plan_errors_match_oracle(name):
    """Chunk-level errors found while walking page headers must be the oracle's (class and page);
    chunks the host accepts must not be chunk-level failures in the oracle."""
    data = pqtest.load(name)
    try:
        plan = _plan_errors(data)
    except pqgpu.DecodeError:
        return  # footer error, covered by test_file_metadata_matches_oracle
    for rg, col, r in pqtest.oracle_decode(data):
        e = plan[(rg, col)]
        if e is not None:
            assert isinstance(r, O.OracleError), (name, rg, col, e)
            assert (e.code, e.page) == (r.code, r.page), (name, rg, col, e, r)


def test_must_not_crash_host():
    """The reference's fuzz regression images through the host planner: footer errors and
    readPages errors match the oracle's class (and page)."""
    d = os.path.join(pqtest.GOLDEN, "must_not_crash")
    for fn in sorted(os.listdir(d)):
        data = open(os.path.join(d, fn), "rb").read()
        try:
            orc = pqtest.oracle_decode(data)
        except O.OracleError as oe:
            with pytest.raises(pqgpu.DecodeError) as ei:
                pqgpu.File(data)
            assert ei.value.code == oe.code, (fn, ei.value, oe)
            continue
        plan = _plan_errors(data)
        for rg, col, r in orc:
            e = plan[(rg, col)]
            if e is not None:
                assert isinstance(r, O.OracleError), (fn, rg, col, e)
                assert (e.code, e.page) == (r.code, r.page), (fn, rg, col, e, r)


def test_ctx_without_gpu_fails_loudly():
    """No silent CPU fallback: without a device the context cannot be created."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    with pytest.raises(pqgpu.DecodeError) as ei:
        pqgpu.Context(0)
    assert ei.value.code == pqgpu.PQ_ERR_HIP
