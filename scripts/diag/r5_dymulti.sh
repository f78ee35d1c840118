#!/bin/bash
# multi-adapter lora_dy (Gemma-3 q|k|v, gate|up): Gemma / LoRA tests, then per-adapter vs multi A/B
set -o pipefail
O=gpurun_out/r5dymulti
mkdir -p $O
export PYTHONPATH=. TMPDIR=/tmp
timeout -k 10 700 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_parity_full_gpu.py tests/test_engine_gpu.py tests/test_lora_dy_gpu.py > $O/tests.txt 2>&1; rc=$?; tail -2 $O/tests.txt; [ $rc -eq 0 ] || { grep -B3 -A30 "Error\|FAIL" $O/tests.txt | head -60; exit 1; }
for r in 1 2; do
  for m in 1 0; do
    MFT_LORA_DY_MULTI=$m timeout -k 10 300 python3 bench.py --config gemma3-270m-lora --steps 20 --warmup 5 > $O/one.txt 2>&1 || { tail -5 $O/one.txt; exit 1; }
    echo "round $r multi=$m $(tail -1 $O/one.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), d["ms_per_step"])')"
  done
done
