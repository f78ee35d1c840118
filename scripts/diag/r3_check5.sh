#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 600 python3 -u -m pytest tests/test_engine_gemma_gpu.py tests/test_engine_gpu.py tests/test_parity_full_gpu.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r3_check5.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "passed|failed" gpurun_out/r3_check5.log | tail -2; grep -E "^FAILED" gpurun_out/r3_check5.log | head; [ $rc -eq 0 ] || exit 1
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --config gemma3-270m-lora --steps 20 --warmup 5 > gpurun_out/r3_c5.json 2> gpurun_out/r3_c5.err || { tail -20 gpurun_out/r3_c5.err; exit 1; }
  echo "gemma: $(python3 -c 'import json; r=json.load(open("gpurun_out/r3_c5.json")); print(r["value"], r["ms_per_step"])')"
done
