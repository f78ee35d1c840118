#!/bin/bash
# LATE phase order as the gemm8 default + per-shape gemm8/hipBLASLt choice for the NT forwards:
# kernel numerics, Python ZeRO-2 chunked reduce-scatter + recorded-RCCL graph tests, then the four
# bench configs (choices printed)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 600 python3 -u -m pytest tests/test_gemm_gpu.py tests/test_lm_head_ce_gpu.py tests/test_dp_graph_gpu.py \
  -q --timeout 240 --timeout-method thread > gpurun_out/r3_ld_tests.log 2>&1; echo "tests rc=$?"
grep -E "passed|failed|Error" gpurun_out/r3_ld_tests.log | tail -5
timeout -k 10 200 python3 scripts/diag/z2_debug.py 2>&1 | grep -v amdgpu.ids | tail -6
MFT_TEST_GRAPH_COMM=1 AMD_LOG_LEVEL=1 timeout -k 10 300 python3 -u -m pytest tests/test_dp_graph_gpu.py -x -v --timeout 240 \
  --timeout-method thread > gpurun_out/r3_graphcomm.log 2>&1; echo "graph-comm tests rc=$?"; grep -E "PASSED|FAILED|rror" gpurun_out/r3_graphcomm.log | tail -12
rm -f gpurun_out/r3_ld_bench.jsonl
for cfg in gpt2-lora gemma3-270m-lora gpt2-full gpt2-xl-zero3; do
  MFT_NT_VERBOSE=1 timeout -k 10 300 python3 bench.py --config $cfg --steps 20 --warmup 5 >> gpurun_out/r3_ld_bench.jsonl 2> gpurun_out/r3_ld_$cfg.err || { tail -20 gpurun_out/r3_ld_$cfg.err; exit 1; }
  echo "$cfg: $(tail -1 gpurun_out/r3_ld_bench.jsonl | cut -c1-220)"
  grep "mft gemm_nt" gpurun_out/r3_ld_$cfg.err | head -12
done
