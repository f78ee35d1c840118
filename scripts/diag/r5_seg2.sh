#!/bin/bash
# LoRA data gradient as a gemm4 second K segment: tests + end-to-end A/B (MFT_LORA_SEG2=0: gemm8 LORA epilogue)
set -o pipefail
O=gpurun_out/${1:-r5o}
mkdir -p $O
export PYTHONPATH=$PWD
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gemm4_gpu.py "tests/test_engine_gpu.py::test_native_cli_matches_python_path" tests/test_parity_full_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
grep -E "passed|failed|vs fp32|rel L2" $O/tests.log | tail -12
: > $O/e2e.txt
one() {  # cfg env
  env $2 timeout -k 10 400 python3 bench.py --config $1 --steps 20 --warmup 5 > $O/one.txt 2>&1 || { tail -20 $O/one.txt; exit 1; }
  echo "$1 $2 $(tail -1 $O/one.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), d["ms_per_step"], d["config"].get("peak_hbm_gb_rank0"))')" | tee -a $O/e2e.txt
}
for r in 1 2; do
  for m in 0 1; do one gpt2-lora MFT_LORA_SEG2=$m || exit 1; done
done
for m in 0 1; do one gemma3-270m-lora MFT_LORA_SEG2=$m || exit 1; done
one gemma3-1b-lora MFT_LORA_SEG2=1 || exit 1
