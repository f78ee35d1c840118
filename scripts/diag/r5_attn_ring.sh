#!/bin/bash
# D = 256 attention forward: ring depth / waves per workgroup / GQA-packed workgroups A/B (gemma3 bench shape)
set -o pipefail
O=gpurun_out/${1:-r5ar}
mkdir -p $O
export PYTHONPATH=.
for v in "4 8 0" "2 8 0" "3 8 0" "2 4 0" "4 4 0" "4 8 1" "2 8 1" "2 4 1" "4 4 1" "4 8 0"; do
  set -- $v
  MFT_ATTN_FWD_RING=$1 MFT_ATTN_NW_FWD=$2 MFT_ATTN_GQA=$3 timeout -k 10 120 python3 scripts/bench_attn256.py >> $O/ring.txt 2>&1 || { tail -5 $O/ring.txt; exit 1; }
done
cat $O/ring.txt
