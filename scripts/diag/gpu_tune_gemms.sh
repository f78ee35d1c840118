#!/bin/bash
# Tune the library GEMM shapes of every bench config with TunableOp (eager warm-up steps only) and
# write the merged database to gpurun_out/tunableop_gfx950.csv (copy into mobilefinetuner_amd/tuning/).
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD MFT_GEMM_TUNE=1 MFT_GEMM_TUNE_DB=$PWD/gpurun_out/tunableop_gfx950.csv
cp mobilefinetuner_amd/tuning/tunableop_gfx950.csv gpurun_out/tunableop_gfx950.csv
for c in ${@:-gpt2-lora gemma3-270m-lora gpt2-full}; do
  timeout -k 10 400 python -u bench.py --config $c --steps 3 --warmup 3 >> gpurun_out/tune.log 2>&1 || { tail gpurun_out/tune.log; exit 1; }
done
wc -l gpurun_out/tunableop_gfx950.csv; tail -3 gpurun_out/tune.log
