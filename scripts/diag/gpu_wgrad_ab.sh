#!/bin/bash
# LoRA weight-gradient kernel A/B (MFMA lora_xty vs VALU lora_wgrad_kernel: MFT_WGRAD_VALU=1), interleaved
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for rep in 1 2; do
for cfg in gemma3-270m-lora gpt2-lora; do
  for V in 0 1; do
    MFT_WGRAD_VALU=$V timeout -k 10 300 python bench.py --config $cfg --steps 15 --warmup 4 > gpurun_out/wg_${cfg}_$V.json 2> gpurun_out/wg_${cfg}_$V.err || { tail -5 gpurun_out/wg_${cfg}_$V.err; exit 1; }
    echo "$cfg VALU=$V $(python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(d['value'], d['ms_per_step'])" gpurun_out/wg_${cfg}_$V.json)"
  done
done
done
