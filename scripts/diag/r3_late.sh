#!/bin/bash
# gemm8 LATE phase order A/B (NT shapes) + the fixed alignment test
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 300 python3 scripts/bench_g8late.py > gpurun_out/r3_g8late.txt 2>&1 || { tail -20 gpurun_out/r3_g8late.txt; exit 1; }
cat gpurun_out/r3_g8late.txt | grep -v amdgpu.ids
timeout -k 10 300 python3 -u -m pytest "tests/test_engine_gemma_gpu.py::test_native_gemma_alignment_harness" -x -q --timeout 240 \
  --timeout-method thread > gpurun_out/r3_align.log 2>&1; tail -3 gpurun_out/r3_align.log
