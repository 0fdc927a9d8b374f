#!/bin/bash
# round 6 session F: copy shapes with unaligned 16-B loads / stores; cfg2 level grid sizes (v1 level kernel)
cd "$GRAFT_REPO_ROOT"
V='[{}, {"PQ_SEG_GRID": 1024}, {"PQ_SEG_GRID": 768}, {"PQ_SEG_GRID": 1536}, {}, {"PQ_SEG_GRID": 1024}]'
tools/gpu_steps.sh \
  "150 copy_shapes tools/ubench/copy_shapes" \
  "300 probe python tools/variant_probe.py --config cfg2 --variants '$V'"
