#!/bin/bash
# Round 5 session 11: full-size verification runs (cfg2, cfg3, cfg4 against the generator's arrays,
# cfg5's resident step against the oracle on sampled chunks).
cd "$(dirname "$0")/.."
B="python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --verify"
tools/gpu_steps.sh \
  "300 s11_verify_cfg4 $B --config cfg4" \
  "300 s11_verify_cfg3 $B --config cfg3" \
  "300 s11_verify_cfg2 $B --config cfg2" \
  "400 s11_verify_cfg5 $B --config cfg5"
