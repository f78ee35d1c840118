#!/bin/bash
# PMC passes over the D=256 attention kernels (one counter group per rocprofv3 run)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp
cd $R
export PYTHONPATH=$R
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT -d gpurun_out/pmc/a1 -o run -- python3 scripts/diag/attn256_pmc_probe.py > gpurun_out/pmc/a1.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT -d gpurun_out/pmc/a2 -o run -- python3 scripts/diag/attn256_pmc_probe.py > gpurun_out/pmc/a2.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum -d gpurun_out/pmc/a3 -o run -- python3 scripts/diag/attn256_pmc_probe.py > gpurun_out/pmc/a3.log 2>&1
rc=$?
for p in a1 a2 a3; do DB=$(find gpurun_out/pmc/$p -name "*.db" | head -1); [ -n "$DB" ] && python3 scripts/pmc_db.py $DB attn_; done > gpurun_out/r3_attn256_pmc.txt
rm -rf gpurun_out/pmc/a1 gpurun_out/pmc/a2 gpurun_out/pmc/a3
cat gpurun_out/r3_attn256_pmc.txt
exit $rc
