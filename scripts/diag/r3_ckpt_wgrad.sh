#!/bin/bash
# activation checkpointing + alignment + Gemma parity tests, then wgrad routing A/B (gemm8 default
# vs MFT_WGRAD=lt hipBLASLt) on gpt2-full and GPT-2 XL ZeRO-3
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 900 python3 -u -m pytest "tests/test_engine_dist_gpu.py::test_native_activation_checkpointing_same_losses" \
  "tests/test_engine_gemma_gpu.py::test_native_gemma_alignment_harness" \
  "tests/test_parity_full_gpu.py::test_gemma3_270m_lora_step_matches_fp32" "tests/test_engine_gpu.py::test_native_weight_streaming_matches_resident" "tests/test_engine_gemma_gpu.py::test_native_gemma_weight_streaming_matches_resident" -v -s --timeout 400 --timeout-method thread > gpurun_out/r3_ckpt.log 2>&1
rc=$?
grep -E "rel L2|loss |PASSED|FAILED|Error" gpurun_out/r3_ckpt.log | tail -30
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
rm -f gpurun_out/r3_wgrad_ab.jsonl
for cfg in gpt2-full gpt2-xl-zero3; do
  for w in gemm8 lt; do
    MFT_WGRAD=$w timeout -k 10 300 python3 bench.py --config $cfg --steps 10 --warmup 3 >> gpurun_out/r3_wgrad_ab.jsonl 2> gpurun_out/r3_wgrad_ab.err || { tail -20 gpurun_out/r3_wgrad_ab.err; exit 1; }
    echo "$cfg wgrad=$w: $(tail -1 gpurun_out/r3_wgrad_ab.jsonl | cut -c1-200)"
  done
done
