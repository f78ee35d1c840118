#!/bin/bash
# gemm8 N-tail quadrant skip A/B (MFT_GEMM8_NTAIL=0 = off), interleaved, Gemma-3 LoRA step
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py tests/test_lm_head_ce_gpu.py > gpurun_out/ntail_tests.log 2>&1 || { tail -30 gpurun_out/ntail_tests.log; exit 1; }
tail -1 gpurun_out/ntail_tests.log
: > gpurun_out/ntail_ab.txt
for r in 1 2; do
  for v in 0 1; do
    out=$(MFT_GEMM8_NTAIL=$v timeout -k 10 300 python3 bench.py --config gemma3-270m-lora --steps 20 --warmup 5 2> gpurun_out/ntail_ab.err) || { tail -5 gpurun_out/ntail_ab.err; exit 1; }
    echo "ntail=$v $(echo "$out" | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')" | tee -a gpurun_out/ntail_ab.txt
  done
done
