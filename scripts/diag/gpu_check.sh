#!/bin/bash
# GPU check used during development: gpu tests, headline bench, GEMM shape sweep.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/bench_default.log 2>&1 && \
timeout -k 10 300 python scripts/bench_gemm.py --M 65536 --bm 8 > gpurun_out/bench_gemm.log 2>&1
rc=$?
tail -3 gpurun_out/gpu_tests.log; tail -1 gpurun_out/bench_default.log; cat gpurun_out/bench_gemm.log
exit $rc
