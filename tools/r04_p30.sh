#!/bin/bash
# Probe: cfg5 with the DELTA pages on their own stream beside the dictionary tiles (PQ_DELTA_SIDE=1).
cd "$(dirname "$0")/.."
exec tools/gpu_steps.sh \
 "300 p_cfg5 python -u tools/variant_probe.py --config cfg5 --variants '[{}, {\"PQ_DELTA_SIDE\": \"1\"}, {}, {\"PQ_DELTA_SIDE\": \"1\"}]'"
