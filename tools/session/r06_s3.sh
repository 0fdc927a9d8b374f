#!/bin/bash
# Round 6 session 3: torn look-back test (readers wait for inclusive prefixes under the injection);
# cfg2 with k_levels_seg as a smaller persistent grid (fewer level waves beside k_values_delta).
cd "$(dirname "$0")/../.."
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
V='[{}, {"PQ_SEG_GRID": "256"}, {"PQ_SEG_GRID": "512"}, {"PQ_SEG_GRID": "1024"}, {"PQ_SEG_GRID": "128"}, {}, {"PQ_SEG_GRID": "256"}, {"PQ_SEG_GRID": "512"}]'
tools/gpu_steps.sh \
  "200 s3_torn $T tests/test_nested.py::test_gpu_lookback_torn_publish tests/test_levels_seg.py -s" \
  "400 s3_probe_seggrid python -u tools/variant_probe.py --config cfg2 --variants '$V'"
