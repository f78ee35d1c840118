# A/B of the LM-head + cross-entropy chunk size (rows per chunk) on the Gemma-3 270M LoRA bench
set -o pipefail
mkdir -p gpurun_out
for c in 512 2048 8192 0; do
  echo "== MFT_CE_CHUNK=$c" >> gpurun_out/b_cechunk.log
  if [ "$c" = 0 ]; then
    timeout -k 10 180 python bench.py --config gemma3-270m-lora --steps 10 --warmup 3 >> gpurun_out/b_cechunk.log 2>&1 || exit 1
  else
    MFT_CE_CHUNK=$c timeout -k 10 180 python bench.py --config gemma3-270m-lora --steps 10 --warmup 3 >> gpurun_out/b_cechunk.log 2>&1 || exit 1
  fi
done
