#!/bin/bash
# gemm4 timing diagnostics (no-memory / no-barrier / no-LDS-DMA variants) + PMC of gemm4 vs gemm8 vs hipBLASLt
set -o pipefail
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp PYTHONPATH=$PWD
MFT_G4_DBG=1 timeout -k 10 240 python3 -u scripts/bench_gemm4.py --rounds 3 --iters 10 --only "fc fwd" > gpurun_out/r3_gemm4_diag.txt 2>&1 || { cat gpurun_out/r3_gemm4_diag.txt; exit 1; }
MFT_G4_DBG=1 timeout -k 10 240 python3 -u scripts/bench_gemm4.py --rounds 3 --iters 10 --only "square" --M 8192 2>&1 | grep square >> gpurun_out/r3_gemm4_diag.txt || exit 1
grep -v amdgpu.ids gpurun_out/r3_gemm4_diag.txt
cd /tmp && cd $GRAFT_REPO_ROOT
true && \
true
rc=$?
for p in g1 g2; do DB=$(find gpurun_out/pmc/$p -name "*.db" | head -1); [ -n "$DB" ] && python3 scripts/pmc_db.py $DB gemm8 gemm4 Cijk; done > gpurun_out/r3_gemm4_pmc.txt
rm -rf gpurun_out/pmc/g1 gpurun_out/pmc/g2
cat gpurun_out/r3_gemm4_pmc.txt
exit $rc
