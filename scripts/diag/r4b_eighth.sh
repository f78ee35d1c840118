#!/bin/bash
# dK/dV kernel on offset pair images (odd rows +544 B, two half-wave DMA ops per piece): numerics, time, PMC
set -o pipefail
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "attn or attention" \
  tests/test_engine_gemma_gpu.py tests/test_parity_full_gpu.py tests/test_lm_head_ce_gpu.py > gpurun_out/r4b8_tests.log 2>&1; rc=$?
tail -2 gpurun_out/r4b8_tests.log
[ $rc -eq 0 ] || { grep -B3 -A25 "Error\|FAIL" gpurun_out/r4b8_tests.log | head -50; exit 1; }
for r in 1 2; do timeout -k 10 120 python3 scripts/bench_attn256.py 2>&1 | grep -v amdgpu.ids || exit 1; done | tee gpurun_out/r4b8_attn.txt
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT -d gpurun_out/pmc/q -o run -- python3 scripts/diag/attn256_pmc_probe.py > gpurun_out/pmc/q.log 2>&1 || exit 1
DB=$(find gpurun_out/pmc/q -name "*.db" | head -1); python3 scripts/pmc_db.py $DB attn_ | tee gpurun_out/r4b8_attn_pmc.txt; rm -rf gpurun_out/pmc/q
timeout -k 10 300 python3 scripts/bench_ce.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r4b8_bench_ce.txt
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --config gemma3-270m-lora --steps 20 --warmup 5 2>/dev/null | tail -1 | cut -c1-160
done
