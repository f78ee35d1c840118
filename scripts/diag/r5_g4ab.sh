#!/bin/bash
# end-to-end A/B of the gemm4 routing (MFT_GEMM4=0 off, 1 = MUL_AUX/dGELU, all = + GELU_D / plain gemm8 calls);
# interleaved rounds on the headline (gpt2-lora) and one round on gemma3-270m-lora
set -o pipefail
mkdir -p gpurun_out
OUT=gpurun_out/${1:-r5_g4ab}.txt
: > $OUT
one() {  # cfg mode
  MFT_GEMM4=$2 timeout -k 10 300 python3 bench.py --config $1 --steps 20 --warmup 5 > gpurun_out/r5_one.txt 2>&1 || { tail -20 gpurun_out/r5_one.txt; exit 1; }
  echo "$1 gemm4=$2 $(tail -1 gpurun_out/r5_one.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), d["ms_per_step"])')" | tee -a $OUT
}
for r in 1 2; do
  for m in 0 1 all; do one gpt2-lora $m || exit 1; done
done
for m in 0 1; do one gemma3-270m-lora $m || exit 1; done
