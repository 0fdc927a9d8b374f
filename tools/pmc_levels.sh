#!/bin/bash
# SQ counter passes over the level kernel (one pass per counter set; each pass its own run).
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc
export PQ_NO_SPEC=1
timeout -s KILL 90 rocprofv3 --kernel-include-regex "k_levels" --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES --output-format csv -d gpurun_out/pmc/p1 -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --rows 16777216 &&
timeout -s KILL 90 rocprofv3 --kernel-include-regex "k_levels" --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_LDS_ATOMIC SQ_BUSY_CYCLES SQ_INSTS_SMEM --output-format csv -d gpurun_out/pmc/p2 -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --rows 16777216
