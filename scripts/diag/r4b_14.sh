#!/bin/bash
# attention output staging at pitch D + 8: numerics, PMC (conflict cycles), time; CE kernels' PMC (the verdict's LM-head
# PMC summary) at the Gemma-3 shape
set -o pipefail
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "attn or attention" \
  tests/test_engine_gemma_gpu.py > gpurun_out/r4b14_tests.log 2>&1; rc=$?
tail -2 gpurun_out/r4b14_tests.log
[ $rc -eq 0 ] || { grep -B3 -A25 "Error\|FAIL" gpurun_out/r4b14_tests.log | head -50; exit 1; }
for r in 1 2; do timeout -k 10 120 python3 scripts/bench_attn256.py 2>&1 | grep -v amdgpu.ids || exit 1; done | tee gpurun_out/r4b14_attn.txt
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT -d gpurun_out/pmc/q -o run -- python3 scripts/diag/attn256_pmc_probe.py > gpurun_out/pmc/q.log 2>&1 || exit 1
DB=$(find gpurun_out/pmc/q -name "*.db" | head -1); python3 scripts/pmc_db.py $DB attn_ | tee gpurun_out/r4b14_attn_pmc.txt; rm -rf gpurun_out/pmc/q
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VALU -d gpurun_out/pmc/c -o run -- python3 scripts/diag/ce_pmc_probe.py > gpurun_out/pmc/c.log 2>&1 || { tail -5 gpurun_out/pmc/c.log; exit 1; }
DB=$(find gpurun_out/pmc/c -name "*.db" | head -1); python3 scripts/pmc_db.py $DB gemm8 ce_ | tee gpurun_out/r4b14_ce_pmc.txt; rm -rf gpurun_out/pmc/c
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT TCC_HIT_sum TCC_MISS_sum -d gpurun_out/pmc/c2 -o run -- python3 scripts/diag/ce_pmc_probe.py > gpurun_out/pmc/c2.log 2>&1 || { tail -5 gpurun_out/pmc/c2.log; exit 1; }
DB=$(find gpurun_out/pmc/c2 -name "*.db" | head -1); python3 scripts/pmc_db.py $DB gemm8 ce_ | tee -a gpurun_out/r4b14_ce_pmc.txt; rm -rf gpurun_out/pmc/c2
