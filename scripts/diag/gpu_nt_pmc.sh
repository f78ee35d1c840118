#!/bin/bash
# two PMC passes over nt_pmc_probe.py (gemm8 NT vs hipBLASLt NT), one counter group per run
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp
cd $R
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY -d gpurun_out/pmc/n1 -o run -- python3 scripts/diag/nt_pmc_probe.py > gpurun_out/pmc/n1.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE GRBM_COUNT -d gpurun_out/pmc/n2 -o run -- python3 scripts/diag/nt_pmc_probe.py > gpurun_out/pmc/n2.log 2>&1
rc=$?
for p in n1 n2; do DB=$(find gpurun_out/pmc/$p -name "*.db" | head -1); [ -n "$DB" ] && python3 scripts/pmc_db.py $DB gemm8 Cijk > gpurun_out/pmc/$p.txt; done
rm -rf gpurun_out/pmc/n1 gpurun_out/pmc/n2
cat gpurun_out/pmc/n1.txt gpurun_out/pmc/n2.txt
exit $rc
