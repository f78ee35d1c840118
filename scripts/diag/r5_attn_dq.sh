#!/bin/bash
# D = 256 attention backward: GQA-packed dQ workgroups A/B (gemma3 bench shape), then the attention GPU tests
set -o pipefail
O=gpurun_out/${1:-r5adq}
mkdir -p $O
export PYTHONPATH=.
for v in "0 8" "1 8" "1 4" "0 4" "0 8" "1 8"; do
  set -- $v
  MFT_ATTN_GQA_DQ=$1 MFT_ATTN_NW_DQ=$2 timeout -k 10 120 python3 scripts/bench_attn256.py >> $O/dq.txt 2>&1 || { tail -5 $O/dq.txt; exit 1; }
done
grep err $O/dq.txt | cut -c1-150
MFT_ATTN_GQA_DQ=1 timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "attention or attn" > $O/tests.txt 2>&1; rc=$?; tail -3 $O/tests.txt; exit $rc
