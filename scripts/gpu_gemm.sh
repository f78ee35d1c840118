#!/bin/bash
# gemm8 layouts: numerics tests + shape sweep vs hipBLASLt
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gemm_tests.log 2>&1
rc=$?
tail -15 gpurun_out/gemm_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u scripts/bench_gemm_t.py > gpurun_out/bench_gemm_t.log 2>&1
rc=$?
cat gpurun_out/bench_gemm_t.log
exit $rc
