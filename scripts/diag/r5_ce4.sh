#!/bin/bash
# gemm4 numerics tests + CE forward on gemm4: tests, CE anatomy g4 vs g8, end-to-end A/B
set -o pipefail
O=gpurun_out/${1:-r5n}
mkdir -p $O
export PYTHONPATH=$PWD
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gemm4_gpu.py tests/test_lm_head_ce_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -2
timeout -k 10 300 python3 scripts/bench_ce.py > $O/ce_g4.txt 2>&1 || { tail -20 $O/ce_g4.txt; exit 1; }
MFT_CE_G4=0 timeout -k 10 300 python3 scripts/bench_ce.py > $O/ce_g8.txt 2>&1 || { tail -20 $O/ce_g8.txt; exit 1; }
echo "== CE g4"; grep -v amdgpu.ids $O/ce_g4.txt; echo "== CE g8"; grep -v amdgpu.ids $O/ce_g8.txt
: > $O/e2e.txt
for r in 1 2; do
  for m in 0 1; do
    MFT_CE_G4=$m timeout -k 10 300 python3 bench.py --config gpt2-lora --steps 20 --warmup 5 > $O/one.txt 2>&1 || { tail -20 $O/one.txt; exit 1; }
    echo "gpt2-lora ce_g4=$m $(tail -1 $O/one.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), d["ms_per_step"])')" | tee -a $O/e2e.txt
  done
done
for m in 0 1; do
  MFT_CE_G4=$m timeout -k 10 300 python3 bench.py --config gemma3-270m-lora --steps 20 --warmup 5 > $O/one.txt 2>&1 || { tail -20 $O/one.txt; exit 1; }
  echo "gemma ce_g4=$m $(tail -1 $O/one.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), d["ms_per_step"])')" | tee -a $O/e2e.txt
done
