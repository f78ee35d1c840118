#!/bin/bash
# short-token GEMM (gemm_s) + seg2 prep trimming: tests, benches incl. the reference recipe (4 x 128)
set -o pipefail
O=gpurun_out/${1:-r5p}
mkdir -p $O
export PYTHONPATH=$PWD
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gemm4_gpu.py "tests/test_engine_gpu.py::test_native_cli_matches_python_path" tests/test_parity_full_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
grep -E "passed|failed|vs fp32" $O/tests.log | tail -4
: > $O/e2e.txt
one() {  # cfg env extra
  env $2 timeout -k 10 400 python3 bench.py --config $1 $3 > $O/one.txt 2>&1 || { tail -20 $O/one.txt; exit 1; }
  echo "$1 $2 $3 $(tail -1 $O/one.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), d["ms_per_step"], d["config"].get("peak_hbm_gb_rank0"))')" | tee -a $O/e2e.txt
}
for m in 0 1; do one gpt2-lora MFT_GEMM_S=$m "--batch 4 --steps 50 --warmup 10" || exit 1; done
for m in 0 1; do one gpt2-lora MFT_GEMM_S=$m "--batch 16 --steps 50 --warmup 10" || exit 1; done
one gpt2-lora MFT_GEMM_S=1 "--steps 20 --warmup 5" || exit 1
one gemma3-270m-lora MFT_GEMM_S=1 "--steps 20 --warmup 5" || exit 1
