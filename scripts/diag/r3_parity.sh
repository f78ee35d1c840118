#!/bin/bash
# full-size fp32 parity (GPT-2-124M LoRA / full, Gemma-3-270M LoRA; Python GPU stack + native CLI),
# the native Gemma alignment harness, then the wgrad / XL NT GEMM shapes (gemm8 vs hipBLASLt)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 900 python3 -u -m pytest tests/test_parity_full_gpu.py "tests/test_engine_gemma_gpu.py::test_native_gemma_alignment_harness" \
  -v -s --timeout 400 --timeout-method thread > gpurun_out/r3_parity.log 2>&1
rc=$?
grep -E "rel L2|loss |PASS|FAIL|Error|error" gpurun_out/r3_parity.log | tail -40
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python3 scripts/bench_wgrad.py > gpurun_out/r3_wgrad.txt 2>&1 || { tail -20 gpurun_out/r3_wgrad.txt; exit 1; }
cat gpurun_out/r3_wgrad.txt
