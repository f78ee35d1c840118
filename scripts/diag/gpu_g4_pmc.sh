#!/bin/bash
# gemm4 PMC passes + a no-memory diagnostic timing (scripts/diag/gemm4_pmc_probe.py, scripts/bench_gemm4.py)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-g4pmc}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
cd $R
S="${2:-8192 8192 8192}"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA SQ_INSTS_LDS GRBM_GUI_ACTIVE GRBM_COUNT -d $O/p1 -o run -- python3 scripts/diag/gemm4_pmc_probe.py $S > $O/p1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr SQ_WAIT_INST_LDS SQ_INSTS_VALU -d $O/p2 -o run -- python3 scripts/diag/gemm4_pmc_probe.py $S > $O/p2.log 2>&1 || exit 1
for p in p1 p2; do DB=$(find $O/$p -name "*.db" | head -1); [ -n "$DB" ] && python3 scripts/pmc_db.py $DB gemm Cijk > $O/$p.txt; done
rm -rf $O/p1 $O/p2
timeout -k 10 120 env MFT_G4_DIAG=nomem python3 scripts/bench_gemm4.py --shapes "8192^3,gpt2 fc fwd" --rounds 3 > $O/nomem.txt 2>&1
