#!/bin/bash
# gemm8 LDS-staged epilogue + first-round stagger A/B; then the DP / Gemma-dump / AMSGrad tests
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 400 python3 scripts/bench_g8_epi.py --rounds 3 > gpurun_out/r4_epi.txt 2>&1 || { tail -30 gpurun_out/r4_epi.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r4_epi.txt
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_engine_dist_gpu.py tests/test_engine_gemma_gpu.py tests/test_kernels_gpu.py -k "two_ranks_match or lora_and_gemma or peer_failure or rccl or embedding_dump or amsgrad" > gpurun_out/r4_dist_tests.log 2>&1; rc=$?
tail -25 gpurun_out/r4_dist_tests.log
exit $rc
