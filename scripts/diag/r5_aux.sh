#!/bin/bash
set -o pipefail
export PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm4_gpu.py 2>&1 | tail -1 || exit 1
timeout -k 10 300 python3 scripts/bench_gemm4.py --epi --shapes "gpt2 fc fwd,gpt2 proj fwd" 2>&1 | grep "|" || exit 1
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/aux.txt 2>&1 || { tail -5 gpurun_out/aux.txt; exit 1; }
  echo "$(tail -1 gpurun_out/aux.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), d["ms_per_step"])')"
done
