#!/bin/bash
# lora_dy with the in-kernel finish: LoRA / engine tests, kernel table, benches
set -o pipefail
O=gpurun_out/r5dyfin
mkdir -p $O
export PYTHONPATH=. TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_lora_dy_gpu.py tests/test_engine_gpu.py tests/test_kernels_gpu.py -k "lora or engine or attn or attention or native" > $O/tests.txt 2>&1; rc=$?; tail -2 $O/tests.txt; [ $rc -eq 0 ] || { grep -B3 -A30 "Error\|FAIL" $O/tests.txt | head -60; exit 1; }
for c in gpt2-lora gemma3-270m-lora gpt2-lora:--batch=4 gpt2-lora gemma3-270m-lora; do
  IFS=: read -r cfg extra <<< "$c"
  timeout -k 10 300 python3 bench.py --config $cfg --steps 20 --warmup 5 $extra > $O/one.txt 2>&1 || { tail -5 $O/one.txt; exit 1; }
  echo "$c $(tail -1 $O/one.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), d["ms_per_step"])')"
done
