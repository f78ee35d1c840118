#!/bin/bash
# attention rework check: all kernel + model GPU tests, then the gpt2-lora / gemma benches
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 600 python3 -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py tests/test_engine_gemma_gpu.py tests/test_parity_full_gpu.py -q --timeout 300 --timeout-method thread \
  > gpurun_out/r3_attnchk_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; grep -E "passed|failed" gpurun_out/r3_attnchk_tests.log | tail -2; grep -E "^FAILED" gpurun_out/r3_attnchk_tests.log | head
[ $rc -eq 0 ] || exit 1
rm -f gpurun_out/r3_attnchk_bench.jsonl
for cfg in gemma3-270m-lora gpt2-lora gemma3-270m-lora; do
  timeout -k 10 300 python3 bench.py --config $cfg --steps 20 --warmup 5 >> gpurun_out/r3_attnchk_bench.jsonl 2> gpurun_out/r3_attnchk_$cfg.err || { tail -20 gpurun_out/r3_attnchk_$cfg.err; exit 1; }
  echo "$cfg: $(tail -1 gpurun_out/r3_attnchk_bench.jsonl | cut -c1-170)"
done
