"""Every schedule / kernel switch the shipped library reads from the environment (host.cpp,
kernels.hip launch_levels) must give the oracle's bytes on every fixture, and its errors at the
same page (the reference's readChunk / readPages / getValuesDecoder path, chunk_reader.go:106-159,
:182-263, :299-362). The default schedule is test_gpu_parity.py; here each alternative is forced:

- PQ_DELTA_TILED=1   DELTA pages through k_delta_walk / k_delta_sums / k_delta_prefix + 2,048-value tiles
- PQ_SPLIT_VALUES=1  the value kernels split over the side stream
- PQ_COPY_MODE=1..3  where k_values_copy waits in the speculative schedule (with PQ_COPY_FUSED=0)
- PQ_COPY_FUSED=0/1  PLAIN / BOOLEAN copies in their own launch, or fused into k_values_delta
- PQ_DELTA_SIDE=1    the DELTA stream in every batch
- PQ_LEVELS_FIRST=1  the level kernels dispatched before the values path
- PQ_NO_SPEC=1       the reference's serial order (levels -> bases -> values)
- PQ_DICT_GROUP=1    at most one dictionary tile per grouped item (with PQ_DICT_PAIR=1)
- PQ_BA_PRESUM=0/1/2 byte-array tile bases by look-back, by the k_ba_sums + k_ba_scan pre-pass, or
                     the pre-pass for the LDS-slot class only
- PQ_LV_WAVE=1       the one-wave level walkers k_levels_bw1w / k_levels_w
- PQ_LV_SEG=0        the list-ranking level kernels everywhere
- PQ_LV_SEGW=1/0     generic level streams by segment speculation (k_levels_segw): all of them, or
                     none (default 2: the definition streams)
- PQ_LV_HYB=0        repetition streams by k_levels' list ranking instead of k_levels_hyb
- PQ_NEST_FUSED=0/1  nested arrays by k_nest_count + k_nest_emit, or by k_nest_tile
- PQ_SCAN_SLOTS=0    byte-array slot tables by their own k_dict_slots launch instead of k_scan_slots
- PQ_LV_SPLIT=0      nested batches' repetition-stream level kernels on the batch stream, not beside
- PQ_NEST_PCOUNT=1   the nested pages' counts by k_nest_pcount, k_nest_tile beside the values path
- PQ_NEST_TCOUNT=1   k_nest_tile's bases from k_nest_tcount + k_nest_scan instead of its look-back
- PQ_SEG_GRID=1/2    k_levels_seg with one / two wavefronts walking every page in turn (the default
                     DELTA-major schedule walks two pages per wave once a batch has over 1,024 pages)
- PQ_COPY_EARLY=0    serial batches' PLAIN copies after k_bases instead of beside the level kernels on
                     counts speculated from the pages' value bytes
- PQ_SCAN_SIDE=0     batches whose DELTA pages run on the batch stream: the run scan and the dictionary
                     tiles after them instead of beside them on the side stream
- PQ_DICT_ONLY=0     dictionary-only batches through the generic speculative schedule (a reset launch
                     per decode) instead of the two-launch one
- PQ_PLAIN_TILE_B=16 PLAIN copy tiles of 16 bytes (2-4 values: every tile boundary moved to a 16-B
                     aligned destination byte, most tiles without a full piece)
"""
import pytest

import pqgpu
import pqtest
import py_oracle as O
from test_gpu_parity import _gpu_decode

pytestmark = pytest.mark.gpu

SWITCHES = {
    "delta_tiled": {"PQ_DELTA_TILED": "1"},
    "split_values": {"PQ_SPLIT_VALUES": "1"},
    "copy_mode1": {"PQ_COPY_FUSED": "0", "PQ_COPY_MODE": "1"},
    "copy_mode2": {"PQ_COPY_FUSED": "0", "PQ_COPY_MODE": "2"},
    "copy_mode3": {"PQ_COPY_FUSED": "0", "PQ_COPY_MODE": "3"},
    "copy_unfused": {"PQ_COPY_FUSED": "0"},
    "copy_fused": {"PQ_COPY_FUSED": "1"},
    "delta_side": {"PQ_DELTA_SIDE": "1"},
    "levels_first": {"PQ_LEVELS_FIRST": "1"},
    "no_spec": {"PQ_NO_SPEC": "1"},
    "dict_group1": {"PQ_DICT_PAIR": "1", "PQ_DICT_GROUP": "1"},
    "ba_presum0": {"PQ_BA_PRESUM": "0"},
    "ba_presum1": {"PQ_BA_PRESUM": "1"},
    "ba_presum2": {"PQ_BA_PRESUM": "2"},
    "lv_wave": {"PQ_LV_WAVE": "1"},
    "lv_listrank": {"PQ_LV_SEG": "0"},
    "lv_segw": {"PQ_LV_SEGW": "1"},
    "lv_segw_none": {"PQ_LV_SEGW": "0"},
    "lv_hyb_off": {"PQ_LV_HYB": "0"},
    "nest_two_pass": {"PQ_NEST_FUSED": "0"},
    "nest_fused": {"PQ_NEST_FUSED": "1"},
    "slots_own_launch": {"PQ_SCAN_SLOTS": "0"},
    "lv_no_split": {"PQ_LV_SPLIT": "0"},
    "nest_pcount": {"PQ_NEST_PCOUNT": "1"},
    "seg_grid1": {"PQ_SEG_GRID": "1"},
    "seg_grid2": {"PQ_SEG_GRID": "2"},
    "plain_tile16": {"PQ_PLAIN_TILE_B": "16"},
    "plain_tile16_unfused": {"PQ_PLAIN_TILE_B": "16", "PQ_COPY_FUSED": "0"},
    "nest_tcount": {"PQ_NEST_TCOUNT": "1"},
    "dict_only_off": {"PQ_DICT_ONLY": "0"},
    "copy_early_off": {"PQ_COPY_EARLY": "0"},
    "scan_side_off": {"PQ_SCAN_SIDE": "0"},
}


@pytest.mark.parametrize("switch", list(SWITCHES))
def test_switch_parity(gpu_ctx, switch, monkeypatch):
    for k, v in SWITCHES[switch].items():
        monkeypatch.setenv(k, v)
    checked = 0
    for name in pqtest.ALL:
        data = pqtest.load(name)
        try:
            orc = pqtest.oracle_decode(data)
        except O.OracleError:
            continue  # footer-level error: no chunk reaches the decoder
        gpu = _gpu_decode(gpu_ctx, data)
        for rg, col, r in orc:
            g = gpu[(rg, col)]
            where = f"{switch} {name} rg{rg} col{col}"
            if isinstance(r, O.OracleError):
                assert isinstance(g, pqgpu.DecodeError), f"{where}: oracle error {r} but GPU decoded"
                assert (g.code, g.page) == (r.code, r.page), f"{where}: {g} vs {r}"
            else:
                assert not isinstance(g, pqgpu.DecodeError), f"{where}: GPU error {g}"
                pqtest.assert_chunk_equal(g, r, where)
            checked += 1
    assert checked > 100
