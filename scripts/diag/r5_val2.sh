#!/bin/bash
# gemm_s 8-wave + packed-fp32 GELU / CE epilogues: tests, kernel times, benches
set -o pipefail
export PYTHONPATH=$PWD
O=gpurun_out/r5s
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm4_gpu.py tests/test_lm_head_ce_gpu.py tests/test_parity_full_gpu.py "tests/test_engine_gpu.py::test_native_cli_matches_python_path" "tests/test_engine_gpu.py::test_native_eager_and_graph_agree" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash scripts/diag/r5_gsprof.sh r5gs2 | grep "gemm_s_kernel\|Cijk" || exit 1
timeout -k 10 300 python3 scripts/bench_gemm4.py --epi --shapes "gpt2 fc fwd,gemma gate|up fwd" > $O/epi.txt 2>&1 || { tail -5 $O/epi.txt; exit 1; }
grep -v amdgpu $O/epi.txt
timeout -k 10 300 python3 scripts/bench_ce.py > $O/ce.txt 2>&1 || { tail -5 $O/ce.txt; exit 1; }
grep "vocab\|CE fwd, no E \|fwd+E+dgrad (auto" $O/ce.txt
for a in "--batch 4 --steps 50 --warmup 10" "--steps 20 --warmup 5" "--config gemma3-270m-lora --steps 20 --warmup 5"; do
  timeout -k 10 300 python3 bench.py $a > $O/one.txt 2>&1 || { tail -5 $O/one.txt; exit 1; }
  echo "$a $(tail -1 $O/one.txt | cut -c1-140)"
done
