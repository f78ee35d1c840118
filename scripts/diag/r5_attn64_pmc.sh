#!/bin/bash
# PMC passes over the GPT-2 short attention kernels (one counter set per run)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5a64pmc
mkdir -p $O
cd /tmp && export TMPDIR=/tmp PYTHONPATH=$R
cd $R && timeout -k 10 120 python3 scripts/diag/attn64_pmc_probe.py 20 > $O/time.txt 2>&1 || { tail -5 $O/time.txt; exit 1; }
cat $O/time.txt
cd /tmp
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT -d $O/p1 -o run -- python3 $R/scripts/diag/attn64_pmc_probe.py 3 > $O/p1.log 2>&1 || { tail -5 $O/p1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_IDX_ACTIVE -d $O/p2 -o run -- python3 $R/scripts/diag/attn64_pmc_probe.py 3 > $O/p2.log 2>&1 || { tail -5 $O/p2.log; exit 1; }
cd $R
for p in p1 p2; do python3 scripts/pmc_db.py $(find $O/$p -name "*.db" | head -1) attn > $O/$p.txt 2>&1 || python3 scripts/pmc_db.py $(find $O/$p -name "*.db" | head -1) > $O/$p.txt 2>&1; cat $O/$p.txt | head -40; done
rm -rf $O/p1 $O/p2
