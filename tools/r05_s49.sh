#!/bin/bash
# Round 5 session 49: k_nest_tile takes counter 0's flags (rep == 0) and the leaf entries' validity
# (def == max_def) from the expansion's equality masks instead of two nest_mask calls (variant library);
# GPU suite on it, cfg4 against the committed build, alternating.
cd "$(dirname "$0")/.."
L=parquet-go-1_amd/lib
B="python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --config cfg4"
tools/gpu_steps.sh \
  "600 s49_gpu_eq env PQGPU_LIB=$L/libpqgpu_eq.so python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -rf" \
  "200 s49_cfg4 $B" \
  "200 s49_cfg4_eq env PQGPU_LIB=$L/libpqgpu_eq.so $B" \
  "200 s49_cfg4_b $B" \
  "200 s49_cfg4_eq_b env PQGPU_LIB=$L/libpqgpu_eq.so $B"
