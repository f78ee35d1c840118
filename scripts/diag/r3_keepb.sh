#!/bin/bash
# gemm8 B0 fragment reuse (KEEPB) A/B on the NT shapes, kernel numerics, then the headline configs
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 300 python3 scripts/bench_g8late.py --variants 3,0 > gpurun_out/r3_keepb.txt 2>&1 || { tail -20 gpurun_out/r3_keepb.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r3_keepb.txt
timeout -k 10 600 python3 -u -m pytest tests/test_gemm_gpu.py tests/test_lm_head_ce_gpu.py tests/test_engine_gpu.py -q --timeout 240 \
  --timeout-method thread > gpurun_out/r3_keepb_tests.log 2>&1; echo "tests rc=$?"
grep -E "passed|failed|Error" gpurun_out/r3_keepb_tests.log | tail -5
rm -f gpurun_out/r3_keepb_bench.jsonl
for cfg in gpt2-lora gemma3-270m-lora gpt2-full; do
  timeout -k 10 300 python3 bench.py --config $cfg --steps 20 --warmup 5 >> gpurun_out/r3_keepb_bench.jsonl 2> gpurun_out/r3_keepb_$cfg.err || { tail -20 gpurun_out/r3_keepb_$cfg.err; exit 1; }
  echo "$cfg: $(tail -1 gpurun_out/r3_keepb_bench.jsonl | cut -c1-200)"
done
