#!/bin/bash
# gemm8 tile-order A/B (MFT_GEMM8_GROUP) on the bench configs, after the GEMM numerics tests
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py tests/test_lm_head_ce_gpu.py > gpurun_out/group_tests.log 2>&1 || { tail -30 gpurun_out/group_tests.log; exit 1; }
tail -2 gpurun_out/group_tests.log
for cfg in gemma3-270m-lora gpt2-lora; do
  for G in 0 4 8 16; do
    MFT_GEMM8_GROUP=$G timeout -k 10 300 python bench.py --config $cfg --steps 15 --warmup 4 > gpurun_out/grp_${cfg}_$G.json 2> gpurun_out/grp_${cfg}_$G.err || { tail -5 gpurun_out/grp_${cfg}_$G.err; exit 1; }
    echo "$cfg G=$G $(python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(d['value'], d['ms_per_step'])" gpurun_out/grp_${cfg}_$G.json)"
  done
done
