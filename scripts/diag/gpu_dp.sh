#!/bin/bash
# DP / ZeRO reducers recorded into the hipGraph (1-rank RCCL), ZeRO-3 graph (copy + aliasing paths);
# ZeRO-2 vs ZeRO-3 benches at N = 1
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_dp_graph_gpu.py "tests/test_models_gpu.py::test_zero3_single_gpu_matches_flat" -x -v --timeout 200 --timeout-method thread > gpurun_out/dp_tests.log 2>&1 || { tail -50 gpurun_out/dp_tests.log; exit 1; }
tail -9 gpurun_out/dp_tests.log
: > gpurun_out/dp_bench.jsonl
for args in "--config gpt2-xl-zero --zero 2" "--config gpt2-xl-zero3" "--config gpt2-xl-zero3-offload"; do
  echo "bench $args"
  timeout -k 10 400 python bench.py $args --steps 10 --warmup 3 >> gpurun_out/dp_bench.jsonl 2> gpurun_out/dp_bench.err || { tail -30 gpurun_out/dp_bench.err; exit 1; }
done
cut -c1-300 gpurun_out/dp_bench.jsonl
