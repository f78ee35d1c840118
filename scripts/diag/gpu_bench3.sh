#!/bin/bash
# full GPU test suite, then the three 1-GPU bench configs
set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_all.log 2>&1 || { tail -40 gpurun_out/gpu_all.log; exit 1; }
tail -3 gpurun_out/gpu_all.log
: > gpurun_out/bench3.jsonl
for c in gpt2-lora gemma3-270m-lora gpt2-full; do
  timeout -k 10 400 python bench.py --config $c --steps 20 --warmup 5 >> gpurun_out/bench3.jsonl 2> gpurun_out/bench3_$c.err || { tail -20 gpurun_out/bench3_$c.err; exit 1; }
done
cat gpurun_out/bench3.jsonl
