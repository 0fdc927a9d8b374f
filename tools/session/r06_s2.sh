#!/bin/bash
# Round 6 session 2: the torn look-back test with its counters in a free slot; cfg2 copy work items
# of 16 KiB / 4 KiB (flat sweep shape of tools/ubench/copy_shapes) fused and unfused.
cd "$(dirname "$0")/../.."
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
V='[{}, {"PQ_PLAIN_TILE_B": "16384"}, {"PQ_PLAIN_TILE_B": "4096"}, {"PQ_PLAIN_TILE_B": "32768"}, {"PQ_PLAIN_TILE_B": "16384", "PQ_COPY_FUSED": "0"}, {"PQ_COPY_FUSED": "0"}, {}, {"PQ_PLAIN_TILE_B": "16384"}]'
tools/gpu_steps.sh \
  "200 s2_torn $T tests/test_nested.py::test_gpu_lookback_torn_publish -s" \
  "400 s2_probe_copytile python -u tools/variant_probe.py --config cfg2 --variants '$V'"
