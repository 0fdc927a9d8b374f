#!/bin/bash
# round 6 session G: PLAIN copy tiles with 16-B aligned inner boundaries, k_values_copy with 4 pieces per
# lane; parity of the value paths, then cfg2 fused / unfused copies x tile sizes x level grid
cd "$GRAFT_REPO_ROOT"
V='[{}, {"PQ_PLAIN_TILE_B": 16384}, {"PQ_PLAIN_TILE_B": 32768}, {"PQ_COPY_FUSED": 0}, {"PQ_COPY_FUSED": 0, "PQ_PLAIN_TILE_B": 16384}, {"PQ_COPY_FUSED": 0, "PQ_PLAIN_TILE_B": 32768}, {"PQ_SEG_GRID": 1024}, {"PQ_SEG_GRID": 1024, "PQ_COPY_FUSED": 0, "PQ_PLAIN_TILE_B": 16384}, {}]'
tools/gpu_steps.sh \
  "400 tests python -u -m pytest tests/test_gpu_parity.py tests/test_switches.py tests/test_refwriter.py tests/test_delta_shapes.py -m gpu -x -q --timeout 120 --timeout-method thread" \
  "300 probe python tools/variant_probe.py --config cfg2 --variants '$V'"
