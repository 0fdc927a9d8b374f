#!/bin/bash
# round 6 session W: phase stamps (diagnostic build, one stream) of cfg4's level kernels and byte-array
# emission, and of cfg3's byte-array emission
cd "$GRAFT_REPO_ROOT"
tools/gpu_steps.sh \
  "200 d4 env PQ_ONE_STREAM=1 python tools/diag_dump.py cfg4" \
  "200 d3 env PQ_ONE_STREAM=1 python tools/diag_dump.py cfg3" \
  "200 d3ba python tools/diag_ba.py cfg3" \
  "200 d4ba env PQ_ONE_STREAM=1 python tools/diag_ba.py cfg4"
