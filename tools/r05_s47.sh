#!/bin/bash
# Round 5 session 47: the 1- / 2-bit SWAR level expansion reading its bits with one unaligned
# 32-bit read (bits25c) instead of bits64c (variant library); GPU suite on it, cfg4 against the
# committed build (SWAR with bits64c), alternating.
cd "$(dirname "$0")/.."
L=parquet-go-1_amd/lib
B="python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --config cfg4"
tools/gpu_steps.sh \
  "600 s47_gpu_b25 env PQGPU_LIB=$L/libpqgpu_b25.so python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -rf" \
  "200 s47_cfg4 $B" \
  "200 s47_cfg4_b25 env PQGPU_LIB=$L/libpqgpu_b25.so $B" \
  "200 s47_cfg4_b $B" \
  "200 s47_cfg4_b25_b env PQGPU_LIB=$L/libpqgpu_b25.so $B"
