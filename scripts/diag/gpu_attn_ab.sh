set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "attention or qknorm" > gpurun_out/t_attn.log 2>&1 || exit 1
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_models_gpu.py > gpurun_out/t_models.log 2>&1 || exit 1
for cfg in "" "MFT_ATTN_NW_DKDV=8" "MFT_ATTN_NW_FWD=4 MFT_ATTN_NW_DQ=4" "MFT_ATTN_V1=1"; do
  echo "== $cfg" >> gpurun_out/b_attn.log
  env $cfg timeout -k 10 180 python bench.py --config gemma3-270m-lora --steps 15 --warmup 4 >> gpurun_out/b_attn.log 2>&1 || exit 1
done
