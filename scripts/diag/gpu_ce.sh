#!/bin/bash
# Fused LM-head CE: numerics tests, then the kernel-level GPU suites and a short headline bench.
set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_lm_head_ce_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/ce_tests.log 2>&1 || { tail -40 gpurun_out/ce_tests.log; exit 1; }
tail -12 gpurun_out/ce_tests.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_all.log 2>&1 || { tail -40 gpurun_out/gpu_all.log; exit 1; }
tail -3 gpurun_out/gpu_all.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/ce_bench.jsonl 2> gpurun_out/ce_bench.err || { tail -20 gpurun_out/ce_bench.err; exit 1; }
cat gpurun_out/ce_bench.jsonl
