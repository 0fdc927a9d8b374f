#!/bin/bash
# Round 5 session 46: SWAR expansion of 1- / 2-bit bit-packed level runs in lf_group_from
# (PQ_LF_SWAR=1 variant library): the whole GPU suite on it, then cfg4 against the default, alternating.
cd "$(dirname "$0")/.."
L=parquet-go-1_amd/lib
B="python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --config cfg4"
tools/gpu_steps.sh \
  "600 s46_gpu_sw env PQGPU_LIB=$L/libpqgpu_sw.so python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -rf" \
  "200 s46_cfg4 $B" \
  "200 s46_cfg4_sw env PQGPU_LIB=$L/libpqgpu_sw.so $B" \
  "200 s46_cfg4_b $B" \
  "200 s46_cfg4_sw_b env PQGPU_LIB=$L/libpqgpu_sw.so $B"
