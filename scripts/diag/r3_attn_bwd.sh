#!/bin/bash
# D=256 attention backward: dK/dV with the Q/dO tile prefetch (LDS-DMA at D=256) and raw barriers in
# the split fwd / dQ loops -- attention numerics, timing (NW A/B for dK/dV), per-kernel stats
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 400 python3 -u -m pytest tests/test_kernels_gpu.py -k "attention" -q --timeout 300 --timeout-method thread \
  > gpurun_out/r3_attnbwd_tests.log 2>&1; rc=$?; echo "attention tests rc=$rc"; grep -E "passed|failed" gpurun_out/r3_attnbwd_tests.log | tail -3
grep -E "^FAILED|Error" gpurun_out/r3_attnbwd_tests.log | head -10
[ $rc -eq 0 ] || exit 1
for nw in 8 4; do
  MFT_ATTN_NW_DKDV=$nw timeout -k 10 120 python3 scripts/bench_attn256.py 2>&1 | grep -v amdgpu.ids | sed "s/^/dkdv NW=$nw: /"
done
for nw in 8 4; do
  rm -rf gpurun_out/p_attn
  MFT_ATTN_NW_DKDV=$nw timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/p_attn -o run -- python3 scripts/bench_attn256.py > gpurun_out/r3_attn_prof.log 2>&1 || { tail gpurun_out/r3_attn_prof.log; exit 1; }
  DB=$(find gpurun_out/p_attn -name "*.db" | head -1)
  echo "== dkdv NW=$nw"; python3 scripts/prof_db.py $DB stats 1 6
done
rm -rf gpurun_out/p_attn
timeout -k 10 300 python3 -u -m pytest tests/test_engine_gemma_gpu.py -x -q --timeout 240 --timeout-method thread > gpurun_out/r3_attn_gemma_tests.log 2>&1; echo "gemma engine tests rc=$?"; tail -2 gpurun_out/r3_attn_gemma_tests.log
timeout -k 10 300 python3 bench.py --config gemma3-270m-lora --steps 20 --warmup 5 > gpurun_out/r3_attn_gemma_bench.jsonl 2> gpurun_out/r3_attn_gemma_bench.err && cut -c1-180 gpurun_out/r3_attn_gemma_bench.jsonl
