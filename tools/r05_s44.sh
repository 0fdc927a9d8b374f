#!/bin/bash
# Round 5 session 44: SQ counters of cfg3's kernels (wave-time breakdown, instruction mix, LDS conflicts).
cd "$(dirname "$0")/.."
tools/gpu_steps.sh \
  "180 s44_pmc_time tools/pmc_pass.sh cfg3 time SQ_WAVES,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_LDS" \
  "180 s44_pmc_mix tools/pmc_pass.sh cfg3 mix SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_LDS,SQ_INSTS_VMEM,SQ_INSTS_BRANCH,SQ_LDS_BANK_CONFLICT,SQ_LDS_IDX_ACTIVE,SQ_WAIT_INST_LDS"
