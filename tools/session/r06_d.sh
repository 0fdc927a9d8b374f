#!/bin/bash
# round 6 session D: cfg2 schedule probes — PLAIN copy tile sizes and level grid sizes (one workload, env
# variants per batch), and the ablation shapes (DELTA pages alone, copies alone, both without levels)
cd "$GRAFT_REPO_ROOT"
V='[{}, {"PQ_PLAIN_TILE_B": 8192}, {"PQ_PLAIN_TILE_B": 16384}, {"PQ_PLAIN_TILE_B": 32768}, {"PQ_SEG_GRID": 512}, {"PQ_SEG_GRID": 1024}, {"PQ_ONE_STREAM": 1}, {"PQ_ONE_STREAM": 1, "PQ_PLAIN_TILE_B": 16384}]'
VS='[{}, {"PQ_PLAIN_TILE_B": 16384}]'
tools/gpu_steps.sh \
  "300 probe python tools/variant_probe.py --config cfg2 --variants '$V'" \
  "200 shape_a python tools/variant_probe.py --config cfg2 --shape a,req --variants '$VS'" \
  "200 shape_b python tools/variant_probe.py --config cfg2 --shape b,req --variants '$VS'" \
  "200 shape_req python tools/variant_probe.py --config cfg2 --shape req --variants '$VS'"
