#!/bin/bash
# D = 256 attention backward: dK/dV ring depth / waves A/B (gemma3 bench shape)
set -o pipefail
O=gpurun_out/${1:-r5akv}
mkdir -p $O
export PYTHONPATH=.
for v in "3 8" "2 8" "2 4" "3 4" "3 8" "2 8"; do
  set -- $v
  MFT_ATTN_DKDV_RING=$1 MFT_ATTN_NW_DKDV=$2 timeout -k 10 120 python3 scripts/bench_attn256.py >> $O/kv.txt 2>&1 || { tail -5 $O/kv.txt; exit 1; }
done
grep err $O/kv.txt | cut -c1-150
