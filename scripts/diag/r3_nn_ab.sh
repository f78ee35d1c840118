#!/bin/bash
# plain NN data-gradient GEMMs: timed gemm8 / hipBLASLt choice vs always gemm8 (interleaved A/B)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
rm -f gpurun_out/r3_nn_ab.jsonl
MFT_NT_VERBOSE=1 timeout -k 10 300 python3 bench.py --config gpt2-full --steps 5 --warmup 3 2>&1 >/dev/null | grep "mft gemm" | sort -u
for cfg in gpt2-full gpt2-lora gemma3-270m-lora; do
  for v in "MFT_NN=gemm8" "MFT_NN=timed" "MFT_NN=gemm8" "MFT_NN=timed"; do
    env $v timeout -k 10 300 python3 bench.py --config $cfg --steps 20 --warmup 5 > gpurun_out/r3_nn_one.json 2> gpurun_out/r3_nn.err || { tail -20 gpurun_out/r3_nn.err; exit 1; }
    echo "$cfg $v $(python3 -c 'import json; r=json.load(open("gpurun_out/r3_nn_one.json")); print(r["value"], r["ms_per_step"])')" | tee -a gpurun_out/r3_nn_ab.txt
  done
done
