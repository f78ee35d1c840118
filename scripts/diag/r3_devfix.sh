#!/bin/bash
# default-device fix check: native engine GPU tests (incl. loopback multi-rank) + smoke + the three native benches
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 600 python3 -u -m pytest tests/test_engine_dist_gpu.py tests/test_engine_gpu.py tests/test_engine_gemma_gpu.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r3d_gpu_tests.log 2>&1; rc=$?; echo "gpu tests rc=$rc"
grep -E "passed|failed" gpurun_out/r3d_gpu_tests.log | tail -2; grep -E "^FAILED" gpurun_out/r3d_gpu_tests.log | head
[ $rc -eq 0 ] || exit 1
rm -f gpurun_out/r3d_bench.jsonl
for cfg in gpt2-lora gemma3-270m-lora gpt2-full; do
  timeout -k 10 300 python3 bench.py --config $cfg --steps 20 --warmup 5 >> gpurun_out/r3d_bench.jsonl 2> gpurun_out/r3d_$cfg.err || { tail -20 gpurun_out/r3d_$cfg.err; exit 1; }
  echo "$cfg: $(tail -1 gpurun_out/r3d_bench.jsonl | cut -c1-170)"
done
