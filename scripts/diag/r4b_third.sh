#!/bin/bash
# rowdot forms A/B + numerics, then the two LoRA benches on the new defaults
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "lora or rowdot" \
  > gpurun_out/r4b3_tests.log 2>&1; rc=$?
tail -2 gpurun_out/r4b3_tests.log
[ $rc -eq 0 ] || exit 1
for r in 1 2; do
  MFT_ROWDOT_V1=1 timeout -k 10 120 python3 scripts/bench_rowdot.py 2>&1 | grep rowdot || exit 1
  timeout -k 10 120 python3 scripts/bench_rowdot.py 2>&1 | grep rowdot || exit 1
done | tee gpurun_out/r4b3_rowdot.txt
for c in gpt2-lora gemma3-270m-lora; do
  timeout -k 10 300 python3 bench.py --config $c --steps 20 --warmup 5 > gpurun_out/r4b3_bench_$c.txt 2>&1 || { tail -5 gpurun_out/r4b3_bench_$c.txt; exit 1; }
  tail -1 gpurun_out/r4b3_bench_$c.txt | cut -c1-200
done
