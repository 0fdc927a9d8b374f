#!/bin/bash
# Round 5 session 43: nested tests on the committed build (back-to-back decodes in every nest mode),
# then SQ counters of cfg4's kernels: the wave-time breakdown and the instruction mix of k_nest_tile.
cd "$(dirname "$0")/.."
tools/gpu_steps.sh \
  "200 s43_nested python -u -m pytest tests/test_nested.py -m gpu -q -x --timeout 120 --timeout-method thread -rf" \
  "60 s43_counters bash -c 'cd /tmp && rocprofv3 -L' " \
  "180 s43_pmc_time tools/pmc_pass.sh cfg4 time SQ_WAVES,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_LDS" \
  "180 s43_pmc_mix tools/pmc_pass.sh cfg4 mix SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_LDS,SQ_INSTS_VMEM,SQ_INSTS_BRANCH,SQ_LDS_BANK_CONFLICT,SQ_LDS_IDX_ACTIVE,SQ_WAIT_INST_LDS"
