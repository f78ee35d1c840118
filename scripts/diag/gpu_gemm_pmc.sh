#!/bin/bash
# PMC passes (one counter group per rocprofv3 run) over scripts/diag/gemm_pmc_probe.py
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp
cd $R
L=${1:-nt,nn,tn}
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAIT_ANY -d gpurun_out/pmc/p1 -o run -- python3 scripts/diag/gemm_pmc_probe.py $L > gpurun_out/pmc/p1.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum -d gpurun_out/pmc/p2 -o run -- python3 scripts/diag/gemm_pmc_probe.py $L > gpurun_out/pmc/p2.log 2>&1
rc=$?
for p in p1 p2; do DB=$(find gpurun_out/pmc/$p -name "*.db" | head -1); [ -n "$DB" ] && python3 scripts/pmc_db.py $DB gemm8; done
rm -rf gpurun_out/pmc/p1 gpurun_out/pmc/p2
exit $rc
