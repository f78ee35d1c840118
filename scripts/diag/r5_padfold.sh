#!/bin/bash
# widened-output zero columns written by the attention / GeGLU kernels: model-level GPU tests + benches
set -o pipefail
O=gpurun_out/r5padfold
mkdir -p $O
export PYTHONPATH=. TMPDIR=/tmp
timeout -k 10 800 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_parity_full_gpu.py tests/test_engine_gpu.py tests/test_kernels_gpu.py tests/test_models_gpu.py > $O/tests.txt 2>&1; rc=$?; tail -2 $O/tests.txt; [ $rc -eq 0 ] || { grep -B3 -A30 "Error\|FAIL" $O/tests.txt | head -60; exit 1; }
for c in gemma3-270m-lora gpt2-lora gemma3-1b-lora; do
  timeout -k 10 300 python3 bench.py --config $c --steps 20 --warmup 5 > $O/one.txt 2>&1 || { tail -5 $O/one.txt; exit 1; }
  echo "$c $(tail -1 $O/one.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), d["ms_per_step"])')"
done
