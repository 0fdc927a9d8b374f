#!/bin/bash
# round 6 session H: cfg2 DELTA launch alone by shape (OPTIONAL vs REQUIRED columns), tile x grid combos
cd "$GRAFT_REPO_ROOT"
V='[{}, {"PQ_SEG_GRID": 1024, "PQ_PLAIN_TILE_B": 32768}, {"PQ_SEG_GRID": 1024, "PQ_PLAIN_TILE_B": 65536}, {"PQ_PLAIN_TILE_B": 65536}, {"PQ_ONE_STREAM": 1}, {"PQ_ONE_STREAM": 1, "PQ_PLAIN_TILE_B": 32768}]'
VS='[{"PQ_ONE_STREAM": 1}, {"PQ_ONE_STREAM": 1, "PQ_PLAIN_TILE_B": 32768}, {"PQ_ONE_STREAM": 1, "PQ_PLAIN_TILE_B": 16384}]'
tools/gpu_steps.sh \
  "300 probe python tools/variant_probe.py --config cfg2 --variants '$V'" \
  "200 shape_a python tools/variant_probe.py --config cfg2 --shape a --variants '$VS'" \
  "200 shape_b python tools/variant_probe.py --config cfg2 --shape b --variants '$VS'" \
  "200 shape_ar python tools/variant_probe.py --config cfg2 --shape a,req --variants '$VS'" \
  "200 shape_br python tools/variant_probe.py --config cfg2 --shape b,req --variants '$VS'"
