# split attention: tests, then the Gemma bench at both dK/dV workgroup sizes, then a kernel profile
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "attention" > gpurun_out/t_attn3.log 2>&1 || exit 1
for cfg in "MFT_ATTN_NW_DKDV=4" "MFT_ATTN_NW_DKDV=8"; do
  echo "== $cfg" >> gpurun_out/b_attn3.log
  env $cfg timeout -k 10 180 python bench.py --config gemma3-270m-lora --steps 15 --warmup 4 >> gpurun_out/b_attn3.log 2>&1 || exit 1
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_gemma4 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config gemma3-270m-lora --steps 5 --warmup 3 > $GRAFT_REPO_ROOT/gpurun_out/p_gemma4.log 2>&1
