#!/bin/bash
# LM-head CE rows per fused call at the 1024 x 128 headline step: 65536 (2 calls) vs 131072 (1 call)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
: > gpurun_out/cechunk_ab.txt
for r in 1 2; do
  for c in 65536 131072; do
    out=$(MFT_CE_CHUNK=$c timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 2> gpurun_out/cechunk_ab.err) || { tail -5 gpurun_out/cechunk_ab.err; exit 1; }
    echo "ce_chunk=$c $(echo "$out" | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')" | tee -a gpurun_out/cechunk_ab.txt
  done
done
