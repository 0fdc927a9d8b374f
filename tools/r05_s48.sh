#!/bin/bash
# Round 5 session 48: compress16 -- the emission's 16-bit validity masks compressed in four rounds
# instead of five (variant library); GPU suite on it, cfg4 against the committed build, alternating.
cd "$(dirname "$0")/.."
L=parquet-go-1_amd/lib
B="python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --config cfg4"
tools/gpu_steps.sh \
  "600 s48_gpu_c16 env PQGPU_LIB=$L/libpqgpu_c16.so python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -rf" \
  "200 s48_cfg4 $B" \
  "200 s48_cfg4_c16 env PQGPU_LIB=$L/libpqgpu_c16.so $B" \
  "200 s48_cfg4_b $B" \
  "200 s48_cfg4_c16_b env PQGPU_LIB=$L/libpqgpu_c16.so $B"
