#!/bin/bash
# LDS-DMA dK/dV kernel: attention tests under every variant, then per-kernel times (rocprofv3
# kernel trace of the attention micro-benchmark at the Gemma-3 shape) for MFT_ATTN_DKDV_DMA=0/2/3
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "attention" > gpurun_out/attn_tests.log 2>&1 || { tail -30 gpurun_out/attn_tests.log; exit 1; }
tail -2 gpurun_out/attn_tests.log
for m in 0 2 3; do
  rm -rf gpurun_out/pa$m
  MFT_ATTN_DKDV_DMA=$m timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/pa$m -o run -- python3 scripts/bench_attn.py --iters 10 > gpurun_out/pa$m.log 2>&1 || { tail gpurun_out/pa$m.log; exit 1; }
  DB=$(find gpurun_out/pa$m -name "*.db" | head -1)
  echo "== MFT_ATTN_DKDV_DMA=$m"; python3 scripts/prof_db.py $DB stats 11 6 | tail -6
  rm -rf gpurun_out/pa$m
done
