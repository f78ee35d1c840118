#!/bin/bash
# D=256 attention forward: 8 waves + 4-slot ring (1 workgroup per CU) vs 4 waves + 2-slot ring (2 per CU)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
MFT_ATTN_FWD_2WG=1 timeout -k 10 300 python3 -u -m pytest tests/test_kernels_gpu.py -k "attention" -x -q --timeout 240 --timeout-method thread > gpurun_out/r3_attn_2wg_tests.log 2>&1; rc=$?
echo "2wg attention tests rc=$rc"; tail -2 gpurun_out/r3_attn_2wg_tests.log; [ $rc -eq 0 ] || exit 1
for n in 0 1 0 1; do MFT_ATTN_FWD_2WG=$n timeout -k 10 120 python3 scripts/bench_attn256.py 2>&1 | grep RPW || exit 1; done
for n in 0 1 0 1; do
  MFT_ATTN_FWD_2WG=$n timeout -k 10 300 python3 bench.py --config gemma3-270m-lora --steps 20 --warmup 5 > gpurun_out/r3_a2_one.json 2> gpurun_out/r3_a2.err || { tail -20 gpurun_out/r3_a2.err; exit 1; }
  echo "gemma 2WG=$n: $(python3 -c 'import json; r=json.load(open("gpurun_out/r3_a2_one.json")); print(r["value"], r["ms_per_step"])')"
done
