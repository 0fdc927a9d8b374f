#!/bin/bash
# round 6 session T: k_ba_emit_slots second slot pieces by LDS-DMA (PQ_BA_DMA=1) against the
# register gathers (libpqgpu_nodma.so), byte-array parity
cd "$GRAFT_REPO_ROOT"
L=$GRAFT_REPO_ROOT/parquet-go-1_amd/lib
tools/gpu_steps.sh \
  "300 tests python -u -m pytest tests/test_ba_classes.py tests/test_gpu_parity.py tests/test_switches.py tests/test_dict_groups.py -m gpu -q -x --timeout 120 --timeout-method thread" \
  "200 c3 python tools/variant_probe.py --config cfg3 --variants '[{}, {}]'" \
  "200 c3nodma env PQGPU_LIB=$L/libpqgpu_nodma.so python tools/variant_probe.py --config cfg3 --variants '[{}, {}]'" \
  "200 c3b python tools/variant_probe.py --config cfg3 --variants '[{}]'"
