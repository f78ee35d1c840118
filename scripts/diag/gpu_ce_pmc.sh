#!/bin/bash
# LM-head CE pieces at the Gemma-3 shape: timings (ce_bench.py) + two PMC passes, one counter group per run
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/cepmc
cd /tmp && export TMPDIR=/tmp
cd $R
export PYTHONPATH=$R
SHAPE="65536 640 262144 262144"
timeout -k 10 200 python3 scripts/diag/ce_bench.py $SHAPE > gpurun_out/cepmc/timing_gemma.txt 2>&1 && cat gpurun_out/cepmc/timing_gemma.txt && \
timeout -k 10 200 python3 scripts/diag/ce_bench.py > gpurun_out/cepmc/timing_gpt2.txt 2>&1 && cat gpurun_out/cepmc/timing_gpt2.txt && \
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY -d gpurun_out/cepmc/p1 -o run -- python3 scripts/diag/ce_bench.py $SHAPE > gpurun_out/cepmc/p1.log 2>&1 && \
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR TCC_EA0_WRREQ_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE -d gpurun_out/cepmc/p2 -o run -- python3 scripts/diag/ce_bench.py $SHAPE > gpurun_out/cepmc/p2.log 2>&1
rc=$?
for p in p1 p2; do DB=$(find gpurun_out/cepmc/$p -name "*.db" | head -1); [ -n "$DB" ] && python3 scripts/pmc_db.py $DB gemm8 Cijk > gpurun_out/cepmc/$p.txt; done
rm -rf gpurun_out/cepmc/p1 gpurun_out/cepmc/p2
cat gpurun_out/cepmc/p1.txt gpurun_out/cepmc/p2.txt 2>/dev/null
exit $rc
