#!/bin/bash
# D=256 attention forward: 8 waves / 128 queries vs 16 waves / 256 queries per workgroup; Gemma CE
# E-buffer budget A/B (32 GB default vs 4 GB: peak HBM and tokens/s)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
MFT_ATTN_FWD_NW=16 timeout -k 10 300 python3 -u -m pytest tests/test_kernels_gpu.py -k "attention" -x -q --timeout 240 --timeout-method thread > gpurun_out/r3_attn_nw16_tests.log 2>&1; rc=$?
echo "nw16 attention tests rc=$rc"; tail -2 gpurun_out/r3_attn_nw16_tests.log; [ $rc -eq 0 ] || exit 1
for n in 8 16 8 16; do MFT_ATTN_FWD_NW=$n timeout -k 10 120 python3 scripts/bench_attn256.py 2>&1 | grep RPW || exit 1; done
rm -f gpurun_out/r3_attn_nw_bench.jsonl
for v in "MFT_ATTN_FWD_NW=8" "MFT_ATTN_FWD_NW=16" "MFT_ATTN_FWD_NW=8 MFT_CE_BUDGET_GB=4" "MFT_ATTN_FWD_NW=16"; do
  env $v timeout -k 10 300 python3 bench.py --config gemma3-270m-lora --steps 20 --warmup 5 >> gpurun_out/r3_attn_nw_bench.jsonl 2> gpurun_out/r3_attn_nw.err || { tail -20 gpurun_out/r3_attn_nw.err; exit 1; }
  echo "$v: $(tail -1 gpurun_out/r3_attn_nw_bench.jsonl | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"], r["config"].get("peak_hbm_gb_rank0"))')"
done
