#!/bin/bash
# gemm4 (4-wave 256x256, AGPR accumulators) correctness + A/B vs gemm8 / hipBLASLt, then the re-entry checks
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 240 python3 -u scripts/bench_gemm4.py --rounds 3 --iters 10 > gpurun_out/r3_gemm4_ab.txt 2>&1; rc=$?
cat gpurun_out/r3_gemm4_ab.txt | grep -v amdgpu.ids
[ $rc -eq 0 ] || exit 1
[ -n "$SKIP_CHECK" ] && exit 0
TESTS="tests/test_models_gpu.py" bash scripts/diag/r3_session_check.sh
