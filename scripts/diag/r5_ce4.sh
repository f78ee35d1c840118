#!/bin/bash
# gemm4 numerics + CE forward on gemm4 + the engine without hipBLASLt: tests, CE anatomy g4 vs g8, benches
set -o pipefail
O=gpurun_out/${1:-r5n}
mkdir -p $O
export PYTHONPATH=$PWD
timeout -k 10 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gemm4_gpu.py tests/test_lm_head_ce_gpu.py "tests/test_engine_gpu.py::test_engine_selftest" "tests/test_engine_gpu.py::test_native_cli_matches_python_path" tests/test_parity_full_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -2
timeout -k 10 300 python3 scripts/bench_ce.py > $O/ce_g4.txt 2>&1 || { tail -20 $O/ce_g4.txt; exit 1; }
MFT_CE_G4=0 timeout -k 10 300 python3 scripts/bench_ce.py > $O/ce_g8.txt 2>&1 || { tail -20 $O/ce_g8.txt; exit 1; }
echo "== CE g4"; grep -v amdgpu.ids $O/ce_g4.txt; echo "== CE g8"; grep -v amdgpu.ids $O/ce_g8.txt
: > $O/e2e.txt
one() {  # cfg env
  env $2 timeout -k 10 400 python3 bench.py --config $1 --steps 20 --warmup 5 > $O/one.txt 2>&1 || { tail -20 $O/one.txt; exit 1; }
  echo "$1 $2 $(tail -1 $O/one.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), d["ms_per_step"], d["config"].get("peak_hbm_gb_rank0"))')" | tee -a $O/e2e.txt
}
for r in 1 2; do
  for m in 0 1; do one gpt2-lora MFT_CE_G4=$m || exit 1; done
done
for m in 0 1; do one gemma3-270m-lora MFT_CE_G4=$m || exit 1; done
one gpt2-full MFT_CE_G4=1 || exit 1
one gpt2-xl-zero3 MFT_CE_G4=1 || exit 1
