#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAIT_ANY -d gpurun_out/pmc/p1 -o run --output-format csv -- python3 scripts/diag/gemm_pmc_probe.py > gpurun_out/pmc/p1.log 2>&1
rc=$?
find gpurun_out/pmc -name "*counter_collection*" | head
exit $rc
