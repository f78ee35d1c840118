#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
MFT_ATTN_RPW=32 timeout -k 10 300 python3 -u -m pytest tests/test_kernels_gpu.py -k "flash_attention or qknorm_rope_attention" -x -q --timeout 240 --timeout-method thread > gpurun_out/r3_attn_tests.log 2>&1; echo "rpw32 attention tests rc=$?"; tail -2 gpurun_out/r3_attn_tests.log
for r in 16 32 16 32; do MFT_ATTN_RPW=$r timeout -k 10 120 python3 scripts/bench_attn256.py 2>&1 | grep RPW; done
timeout -k 10 200 python3 scripts/diag/z2_debug.py 2>&1 | grep -v amdgpu.ids | grep -E "mismatch|rel diff|sync" | tail -8
