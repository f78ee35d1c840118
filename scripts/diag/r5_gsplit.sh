#!/bin/bash
# gemm_s split-K across workgroups: tests, short-token shape timings and the 4 x 128 recipe, split on / off
set -o pipefail
O=gpurun_out/${1:-r5gsplit}
mkdir -p $O
export PYTHONPATH=. TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm4_gpu.py > $O/tests.txt 2>&1; rc=$?; tail -2 $O/tests.txt; [ $rc -eq 0 ] || { grep -B3 -A30 "Error\|FAIL" $O/tests.txt | head -60; exit 1; }
for sp in 0 1 0 1; do
  MFT_GS_SPLIT=$sp timeout -k 10 200 python3 scripts/bench_gemm4.py --shapes "b4 proj fwd,b4 fc fwd,b4 mproj fwd" --rounds 3 --iters 20 --only gemm_s > $O/sh_$sp.txt 2>&1 || { tail -5 $O/sh_$sp.txt; exit 1; }
  echo "split=$sp"; cat $O/sh_$sp.txt | cut -c1-110
done
for sp in 0 1 0 1; do
  MFT_GS_SPLIT=$sp timeout -k 10 300 python3 bench.py --config gpt2-lora --batch 4 --steps 50 --warmup 10 > $O/b4_$sp.txt 2>&1 || { tail -5 $O/b4_$sp.txt; exit 1; }
  echo "b4 split=$sp: $(tail -1 $O/b4_$sp.txt | cut -c1-120)"
done
