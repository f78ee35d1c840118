#!/bin/bash
# end-to-end A/B: plain NT / W^T data-grad GEMMs on gemm4 (default) vs hipBLASLt (MFT_NT=lt), interleaved
set -o pipefail
mkdir -p gpurun_out
OUT=gpurun_out/${1:-r5_ntab}.txt
: > $OUT
one() {  # cfg nt
  MFT_NT=$2 timeout -k 10 300 python3 bench.py --config $1 --steps 20 --warmup 5 > gpurun_out/r5_one.txt 2>&1 || { tail -20 gpurun_out/r5_one.txt; exit 1; }
  echo "$1 nt=$2 $(tail -1 gpurun_out/r5_one.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), d["ms_per_step"])')" | tee -a $OUT
}
for r in 1 2; do
  for m in lt gemm4; do one gpt2-lora $m || exit 1; done
done
for m in lt gemm4; do one gemma3-270m-lora $m || exit 1; done
for m in lt gemm4; do one gpt2-full $m || exit 1; done
