#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 400 python3 -u -m pytest tests/test_engine_gpu.py tests/test_lm_head_ce_gpu.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r3_check4.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "passed|failed" gpurun_out/r3_check4.log | tail -2; grep -E "^FAILED" gpurun_out/r3_check4.log | head; [ $rc -eq 0 ] || exit 1
bash scripts/diag/r3_gemma_prof.sh > /dev/null || exit 1
grep "ce_finalize\|sum_rows\|count_valid\|total GPU" gpurun_out/r3_native_gemma_kernel_stats.txt gpurun_out/r3_native_gpt2_kernel_stats.txt | cut -c1-150
