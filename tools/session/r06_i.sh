#!/bin/bash
# round 6 session I: the GPU suite and smoke on the current build (unaligned DELTA output stores, unzeroed
# validity bitmaps of whole-word k_levels_seg chunks), then cfg2 probes: DELTA at 6 waves per SIMD, tiles x grid
cd "$GRAFT_REPO_ROOT"
L=$GRAFT_REPO_ROOT/parquet-go-1_amd/lib
V='[{}, {"PQ_PLAIN_TILE_B": 32768}, {"PQ_SEG_GRID": 1024}, {"PQ_SEG_GRID": 1024, "PQ_PLAIN_TILE_B": 32768}, {"PQ_ONE_STREAM": 1}, {}]'
tools/gpu_steps.sh \
  "700 tests python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "120 smoke python -c 'import __graft_entry__ as g; g.smoke()'" \
  "300 probe python tools/variant_probe.py --config cfg2 --variants '$V'" \
  "300 probe_wpe6 env PQGPU_LIB=$L/libpqgpu_wpe6.so python tools/variant_probe.py --config cfg2 --variants '$V'"
