#!/bin/bash
# lora_dy / lora_xty block-count A/B (MFT_DY_BLOCKS) on both LoRA bench configs, after the LoRA kernel tests
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest -x -q --timeout 120 --timeout-method thread tests/test_lora_dy_gpu.py tests/test_lora_wgrad_gpu.py > gpurun_out/dy_tests.log 2>&1 || { tail -20 gpurun_out/dy_tests.log; exit 1; }
tail -1 gpurun_out/dy_tests.log
for rep in 1 2; do
for cfg in gemma3-270m-lora gpt2-lora; do
  for NB in 512 1024 2048; do
    MFT_DY_BLOCKS=$NB timeout -k 10 300 python bench.py --config $cfg --steps 15 --warmup 4 > gpurun_out/dy_${cfg}_$NB.json 2> gpurun_out/dy_${cfg}_$NB.err || { tail -5 gpurun_out/dy_${cfg}_$NB.err; exit 1; }
    echo "$cfg NB=$NB $(python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(d['value'], d['ms_per_step'])" gpurun_out/dy_${cfg}_$NB.json)"
  done
done
done
