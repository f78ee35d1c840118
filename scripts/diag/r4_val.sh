#!/bin/bash
# round-4 validation: engine self-test (fused norm + LoRA u), native parity / dist / Gemma / AMSGrad
# tests, then the headline + Gemma + XL ZeRO-3 host-streamed offload benches
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
MODE=${1:-all}
if [ "$MODE" != bench ]; then
timeout -k 10 300 mobilefinetuner_amd/bin/engine_selftest > gpurun_out/r4_selftest.log 2>&1; rc=$?
grep -E "fused LoRA|FAIL|ALL OK" gpurun_out/r4_selftest.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 1500 python -u -m pytest --maxfail 4 -v --timeout 300 --timeout-method thread tests/test_engine_gpu.py \
  tests/test_engine_gemma_gpu.py tests/test_engine_dist_gpu.py tests/test_kernels_gpu.py -k "not lm_head_ce_big" \
  > gpurun_out/r4_val_tests.log 2>&1; rc=$?
tail -15 gpurun_out/r4_val_tests.log
[ $rc -eq 0 ] || exit 1
fi
[ "$MODE" = tests ] && exit 0
for c in gpt2-lora gemma3-270m-lora gpt2-xl-zero3-offload; do
  timeout -k 10 400 python3 bench.py --config $c --steps 20 --warmup 5 > gpurun_out/r4_val_bench_$c.txt 2>&1 || { tail -5 gpurun_out/r4_val_bench_$c.txt; exit 1; }
  tail -1 gpurun_out/r4_val_bench_$c.txt | cut -c1-400
done
timeout -k 10 400 python3 bench.py --config gpt2-xl-zero3-offload --offload_fp32 --steps 10 --warmup 3 > gpurun_out/r4_val_bench_xl_fp32.txt 2>&1 || { tail -5 gpurun_out/r4_val_bench_xl_fp32.txt; exit 1; }
tail -1 gpurun_out/r4_val_bench_xl_fp32.txt | cut -c1-400
