#!/bin/bash
# residual-producing projections on gemm8 (BIAS_ADD, default) vs hipBLASLt beta = 1 (MFT_RESID_LT=1): numerics + A/B
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 900 python -u -m pytest --maxfail 4 -q --timeout 300 --timeout-method thread tests/test_engine_gpu.py \
  tests/test_parity_full_gpu.py > gpurun_out/r4b13_tests.log 2>&1; rc=$?
tail -2 gpurun_out/r4b13_tests.log
[ $rc -eq 0 ] || { grep -A3 "^FAILED\|AssertionError" gpurun_out/r4b13_tests.log | head -40; exit 1; }
for r in 1 2 3; do
  for e in MFT_RESID_LT=0 MFT_RESID_LT=1; do
    for c in gpt2-lora gpt2-full; do
      line=$(env $e timeout -k 10 300 python3 bench.py --config $c --steps 20 --warmup 5 2>/dev/null | tail -1) || { echo "FAIL $c $e"; exit 1; }
      echo "$c [$e]: $(echo "$line" | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print(r['value'], r['ms_per_step'])")"
    done
  done
done | tee gpurun_out/r4b13_ab.txt
