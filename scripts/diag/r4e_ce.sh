#!/bin/bash
# CE-forward epilogue change (padding mask folded into the max pass, v_max3 chain): numerics + timing
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=.
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_lm_head_ce_gpu.py > gpurun_out/r4e_ce_tests.txt 2>&1 &&
timeout -k 10 300 python -u scripts/bench_ce.py --rounds 3 --iters 5 > gpurun_out/r4e_bench_ce.txt 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r4e_bench.txt 2>&1
