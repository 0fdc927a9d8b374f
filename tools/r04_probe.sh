#!/bin/bash
# Round-4 probe session (one gpurun call): level-kernel parity, cfg2 schedule probe and phase
# stamps, cfg4 byte-array base variants; each step under its own limit (tools/gpu_steps.sh).
cd "$(dirname "$0")/.."
exec tools/gpu_steps.sh \
  "300 t_seg python -u -m pytest tests/test_levels_seg.py tests/test_levels_segw.py tests/test_nested.py tests/test_struct.py tests/test_gpu_parity.py tests/test_refwriter.py tests/test_ref_goldens.py tests/test_ba_classes.py tests/test_plain_bytearray.py tests/test_delta_bytearray.py tests/test_stride.py tests/test_snappy.py -m gpu -x -q --timeout 120 --timeout-method thread" \
  "200 probe_cfg2 python -u tools/variant_probe.py --config cfg2 --variants '[{}, {\"PQ_SPEC\": \"0\", \"PQ_SPLIT_VALUES\": \"1\", \"PQ_COPY_FUSED\": \"1\"}]'" \
  "120 diag_cfg2 env PQ_SPEC=0 python -u tools/diag.py cfg2" \
  "200 probe_cfg4 python -u tools/variant_probe.py --config cfg4 --variants '[{}, {\"PQ_BA_PRESUM\": \"1\"}, {\"PQ_BA_PRESUM\": \"2\"}, {\"PQ_LV_SEG\": \"0\"}]'" \
  "200 probe_cfg3 python -u tools/variant_probe.py --config cfg3 --variants '[{}]'" \
  "200 probe_cfg3_nop0 env PQGPU_LIB=$PWD/parquet-go-1_amd/lib/libpqgpu_nop0.so python -u tools/variant_probe.py --config cfg3 --variants '[{}]'" \
  "300 probe_cfg5 python -u tools/variant_probe.py --config cfg5 --variants '[{}]'" \
  "300 probe_cfg5_noldict env PQGPU_LIB=$PWD/parquet-go-1_amd/lib/libpqgpu_noldict.so python -u tools/variant_probe.py --config cfg5 --variants '[{}]'" \
  "$@"
