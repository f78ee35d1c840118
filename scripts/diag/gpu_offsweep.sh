#!/bin/bash
# host-offloaded AdamW: chunk size x device slots sweep (GPT-2 XL ZeRO-3, bf16 moments)
set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
: > gpurun_out/offsweep.txt
for cs in "33554432 2" "33554432 3" "67108864 2" "16777216 2" "67108864 3"; do
  set -- $cs
  MFT_OFFLOAD_CHUNK=$1 MFT_OFFLOAD_SLOTS=$2 timeout -k 10 300 python bench.py --config gpt2-xl-zero3-offload --steps 8 --warmup 3 2>>gpurun_out/offsweep.err | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('chunk $1 slots $2', d['ms_per_step'])" >> gpurun_out/offsweep.txt || exit 1
  tail -1 gpurun_out/offsweep.txt
done
