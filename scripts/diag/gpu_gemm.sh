#!/bin/bash
# gemm8 layouts: numerics tests + shape sweep vs hipBLASLt (persistent and one-tile-per-WG forms)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gemm_tests.log 2>&1
rc=$?
tail -15 gpurun_out/gemm_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u scripts/bench_gemm_t.py ${GEMM_ONLY:+--only "$GEMM_ONLY"} > gpurun_out/bench_gemm_t.log 2>&1 || exit 1
MFT_GEMM8_PERSISTENT=0 timeout -k 10 400 python -u scripts/bench_gemm_t.py ${GEMM_ONLY:+--only "$GEMM_ONLY"} > gpurun_out/bench_gemm_t_np.log 2>&1 || exit 1
echo "== persistent"; cat gpurun_out/bench_gemm_t.log; echo "== one tile per WG"; cat gpurun_out/bench_gemm_t_np.log
