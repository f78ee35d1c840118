#!/bin/bash
# headline CE row chunking A/B: default (4 GiB -> 42688-row chunks: 3 full + one of 3008 rows), balanced 4 x 32768,
# 3 x 43776 (4.1 GiB), 2 x 65536 (6.1 GiB); interleaved rounds
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/r4h_chunk.txt
for r in 1 2 3; do
  for ch in 0 32768 43776 65536; do
    if [ $ch -eq 0 ]; then unset MFT_CE_CHUNK; else export MFT_CE_CHUNK=$ch; fi
    timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r4h_one.txt 2>&1 || { tail -5 gpurun_out/r4h_one.txt; exit 1; }
    echo "round $r chunk $ch $(tail -1 gpurun_out/r4h_one.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), d["ms_per_step"], d["config"].get("peak_hbm_gb_rank0"))')" | tee -a gpurun_out/r4h_chunk.txt
  done
done
