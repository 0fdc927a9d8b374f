"""Byte-array emit paths (bytearray.hip): dictionary entries of 0-12 / 13-28 bytes (16/32-byte
slot tables, k_ba_emit_slots), 29-60 bytes (64-byte slots, k_ba_emit_slots64), longer entries
(no slot table) and a dictionary chunk that falls back to PLAIN pages (k_ba_emit: slot and
source paths in one chunk), each over several row groups and pages of many 4096-value tiles so
the payload-base look-back crosses tiles, pages and queues. Values are known to the generator
(type_dict.go:40-60 gather, type_bytearray.go:24-55 PLAIN); the oracle must return them and the
GPU must equal the oracle."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import rawpq  # noqa: E402

import pqtest  # noqa: E402
import py_oracle as O  # noqa: E402

COLS = {"s12": (0, 12), "s28": (13, 28), "s60": (29, 60), "s200": (0, 200), "mix": (0, 28)}
PAGE_ROWS = [20000, 4096, 1, 9000]


def _vocab(rng, k, lo, hi):
    out = set()
    while len(out) < k:
        out.add(bytes(rng.integers(0, 256, int(rng.integers(lo, hi + 1)), dtype=np.uint8)))
    return sorted(out)


def build(seed=0, row_groups=3):
    rng = np.random.default_rng(700 + seed)
    n = sum(PAGE_ROWS)
    names = list(COLS)
    expect = {name: [] for name in names}
    rgs = []
    for _ in range(row_groups):
        chunks = []
        for name in names:
            lo, hi = COLS[name]
            vocab = _vocab(rng, 1000, lo, hi)
            idx = rng.integers(0, len(vocab), n)
            nulls = rng.random(n) < 0.1
            dl = (~nulls).astype(int).tolist()
            pages = [rawpq.dict_page_ref("BYTE_ARRAY", vocab)]
            at = 0
            for k, pr in enumerate(PAGE_ROWS):
                sl = slice(at, at + pr)
                at += pr
                nn = idx[sl][~nulls[sl]]
                if name == "mix" and k >= 2:  # dictionary overflow: the writer continues PLAIN
                    body, enc = rawpq.plain_encode("BYTE_ARRAY", [vocab[i] for i in nn]), "PLAIN"
                else:
                    body, enc = rawpq.dict_values_section(nn, len(vocab)), "RLE_DICTIONARY"
                pages.append(rawpq.data_page_v1_ref(pr, enc, body, dl[sl], 1))
            expect[name].append(([vocab[i] for i in idx[~nulls]], np.array(dl)))
            chunks.append((pages, n, True))
        rgs.append((n, chunks))
    schema = [[(4, rawpq.BIN, "schema"), (5, rawpq.I32, len(names))]]
    schema += [rawpq.schema_leaf(name, "BYTE_ARRAY", "OPTIONAL") for name in names]
    leaves = [(name, "BYTE_ARRAY") for name in names]
    return rawpq.write_file_schema(schema, leaves, rgs), expect


def test_oracle_ba_classes():
    data, expect = build()
    f = O.File(data)
    for rg in range(3):
        for c, name in enumerate(COLS):
            r = f.read_chunk(rg, c)
            ev, dl = expect[name][rg]
            np.testing.assert_array_equal(r.def_levels, dl, err_msg=name)
            assert pqtest.oracle_values(r) == ev, (rg, name)


# Class routing (host.cpp): the 1,000-entry dictionaries of 16/32-B slots go to class 3 (first slot
# pieces in LDS) by default, and to class 0 (k_ba_emit_slots: slot gathers) without it.
BA_ROUTES = {"default": {}, "gather": {"PQ_BA_LDS_SLOTS": "0"}}


def set_route(monkeypatch, route):
    for k, v in BA_ROUTES[route].items():
        monkeypatch.setenv(k, v)


@pytest.mark.gpu
@pytest.mark.parametrize("route", list(BA_ROUTES))
@pytest.mark.parametrize("seed", [0, 1])
def test_gpu_ba_classes(gpu_ctx, seed, route, monkeypatch):
    import test_gpu_parity as P
    set_route(monkeypatch, route)
    data, _ = build(seed)
    gpu = P._gpu_decode(gpu_ctx, data)
    for rg, col, r in pqtest.oracle_decode(data):
        pqtest.assert_chunk_equal(gpu[(rg, col)], r, f"seed={seed} {route} rg{rg} {list(COLS)[col]}")


HELP_SCRIPT = r"""
import os, sys
sys.path[:0] = sys.argv[1:4]
import test_ba_classes as T, test_gpu_parity as P, pqtest, pqgpu
data, _ = T.build(0, row_groups=2)
gpu = P._gpu_decode(pqgpu.Context(0), data)
for rg, col, r in pqtest.oracle_decode(data):
    pqtest.assert_chunk_equal(gpu[(rg, col)], r, f"help rg{rg} col{col}")
print("HELP-OK")
"""


@pytest.mark.gpu
def test_gpu_lookback_self_help():
    """Every predecessor treated as silent (diagnostic library, PQ_ABLATE bit 12): each tile's
    payload base comes from tile_aggregate alone and must give the same outputs."""
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    diag = os.path.join(root, "parquet-go-1_amd", "lib", "libpqgpu_diag.so")
    assert os.path.exists(diag), "make -C parquet-go-1_amd diag"
    env = dict(os.environ, PQGPU_LIB=diag, PQ_ABLATE=str(1 << 12))
    tests = os.path.dirname(os.path.abspath(__file__))
    r = subprocess.run([sys.executable, "-c", HELP_SCRIPT, tests, os.path.join(root, "parquet-go-1_amd"),
                        os.path.join(root, "oracle")],
                       env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0 and "HELP-OK" in r.stdout, r.stdout[-2000:] + r.stderr[-2000:]


@pytest.mark.gpu
@pytest.mark.parametrize("route", list(BA_ROUTES))
@pytest.mark.parametrize("name", ["cfg3_small", "cfg3_dict64k", "types_dict", "bad_dict_index", "cfg4_small"])
def test_gpu_ba_routes_goldens(gpu_ctx, name, route, monkeypatch):
    """The byte-array goldens (cfg3_dict64k: SURVEY.md §8(d)'s 65,536-entry, 16-bit dictionary)
    through every k_ba_emit route: the oracle's bytes, or its error at the same page."""
    import test_gpu_parity as P
    set_route(monkeypatch, route)
    data = pqtest.load(name)
    gpu = P._gpu_decode(gpu_ctx, data)
    for rg, col, r in pqtest.oracle_decode(data):
        g = gpu[(rg, col)]
        where = f"{name} {route} rg{rg} col{col}"
        if isinstance(r, O.OracleError):
            assert isinstance(g, P.pqgpu.DecodeError), f"{where}: oracle error {r} but GPU decoded"
            assert (g.code, g.page) == (r.code, r.page), f"{where}: {g} vs {r}"
        else:
            assert not isinstance(g, P.pqgpu.DecodeError), f"{where}: GPU error {g}"
            pqtest.assert_chunk_equal(g, r, where)
