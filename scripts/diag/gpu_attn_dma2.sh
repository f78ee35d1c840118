# two-query-group DMA forward (MFT_ATTN_DMA=2): tests under it, micro-bench 1 vs 2, Gemma bench
set -o pipefail
mkdir -p gpurun_out
MFT_ATTN_DMA=2 timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "attention" > gpurun_out/t_dma2.log 2>&1 || exit 1
timeout -k 10 120 python3 scripts/bench_attn.py > gpurun_out/attn_dma1.log 2>&1 || exit 1
MFT_ATTN_DMA=2 timeout -k 10 120 python3 scripts/bench_attn.py > gpurun_out/attn_dma2.log 2>&1 || exit 1
MFT_ATTN_DMA=2 timeout -k 10 180 python bench.py --config gemma3-270m-lora --steps 15 --warmup 4 > gpurun_out/b_dma2.log 2>&1 || exit 1
