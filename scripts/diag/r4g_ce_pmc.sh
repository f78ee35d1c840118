#!/bin/bash
# CE kernels' PMC at the Gemma-3 shape after the round-4 CE-forward epilogue change (VALU per MFMA)
set -o pipefail
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VALU -d gpurun_out/pmc/c -o run -- python3 scripts/diag/ce_pmc_probe.py > gpurun_out/pmc/c.log 2>&1 || { tail -5 gpurun_out/pmc/c.log; exit 1; }
DB=$(find gpurun_out/pmc/c -name "*.db" | head -1); python3 scripts/pmc_db.py $DB gemm8 ce_ | tee gpurun_out/r4g_ce_pmc.txt; rm -rf gpurun_out/pmc/c
