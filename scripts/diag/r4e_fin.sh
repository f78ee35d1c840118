#!/bin/bash
# ce_finalize rows-per-block change: CE numerics, Gemma-3 / GPT-2 bench, Gemma graph kernel table
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=.
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_lm_head_ce_gpu.py > gpurun_out/r4e_fin_tests.txt 2>&1 &&
timeout -k 10 400 python -u bench.py --config gemma3-270m-lora --steps 20 --warmup 5 > gpurun_out/r4e_bench_gemma.txt 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r4e_bench_gpt2.txt 2>&1 &&
bash scripts/diag/r4_gprof.sh > gpurun_out/r4e_gprof.txt 2>&1
