#!/bin/bash
# zero-copy vs streamed optimizer offload: tests, GPT-2 XL ZeRO-3 offload benches, sharding A/B
set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_models_gpu.py -k "offload" -x -v --timeout 120 --timeout-method thread > gpurun_out/zc_tests.log 2>&1 || { tail -40 gpurun_out/zc_tests.log; exit 1; }
tail -7 gpurun_out/zc_tests.log
: > gpurun_out/zc_bench.txt
for m in zerocopy stream; do
  MFT_OFFLOAD_MODE=$m timeout -k 10 300 python bench.py --config gpt2-xl-zero3-offload --steps 8 --warmup 3 2>>gpurun_out/zc_bench.err | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$m', d['ms_per_step'], d['value'])" >> gpurun_out/zc_bench.txt || exit 1
  tail -1 gpurun_out/zc_bench.txt
done
MFT_OFFLOAD_MODE=zerocopy timeout -k 10 300 python bench.py --config gpt2-xl-zero3-offload --offload_fp32 --steps 8 --warmup 3 2>>gpurun_out/zc_bench.err | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('zerocopy fp32', d['ms_per_step'], d['value'])" >> gpurun_out/zc_bench.txt && tail -1 gpurun_out/zc_bench.txt
timeout -k 10 600 python scripts/bench_memory.py sharding --steps 20 --out gpurun_out/shard_ab.jsonl > gpurun_out/shard_ab.log 2>&1 || { tail -20 gpurun_out/shard_ab.log; exit 1; }
cut -c1-200 gpurun_out/shard_ab.jsonl
