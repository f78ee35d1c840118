#!/bin/bash
# optimizer offload (bf16 / fp32 moments), sharder, ZeRO / DP graph tests; offload + ZeRO benches
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_models_gpu.py tests/test_dp_graph_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/off_tests.log 2>&1 || { tail -50 gpurun_out/off_tests.log; exit 1; }
tail -4 gpurun_out/off_tests.log
: > gpurun_out/off_bench.jsonl
for args in "--config gpt2-xl-zero3-offload" "--config gpt2-xl-zero3-offload --offload_fp32" "--config gpt2-xl-zero3"; do
  echo "bench $args"
  timeout -k 10 400 python bench.py $args --steps 10 --warmup 3 >> gpurun_out/off_bench.jsonl 2> gpurun_out/off_bench.err || { tail -30 gpurun_out/off_bench.err; exit 1; }
done
cut -c1-330 gpurun_out/off_bench.jsonl
