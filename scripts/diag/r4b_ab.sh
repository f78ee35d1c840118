#!/bin/bash
# round 4 A/B, interleaved rounds: the LM-head E-buffer budget now that a short row chunk's CE dgrad
# splits the vocab (MFT_CE_BUDGET_GB 32 = one 65536-row chunk vs 4 / 2 GB), and gemm8's LDS-staged
# epilogues (MFT_GEMM8_STREAM=5) vs the register epilogue, on Gemma-3 and the GPT-2 headline
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
out=gpurun_out/r4b_ab.txt; : > $out
run() {  # cfg, env...
  local cfg=$1; shift
  line=$(env "$@" timeout -k 10 300 python3 bench.py --config $cfg --steps 15 --warmup 5 2>/dev/null | tail -1) || { echo "FAIL $cfg $*" | tee -a $out; exit 1; }
  v=$(echo "$line" | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print(r['value'], r['ms_per_step'], r['config'].get('peak_hbm_gb_rank0'))")
  echo "$cfg [$*]: $v" | tee -a $out
}
timeout -k 10 300 python3 scripts/bench_ce.py > gpurun_out/r4b_bench_ce.txt 2>&1 || { tail -20 gpurun_out/r4b_bench_ce.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r4b_bench_ce.txt
for r in 1 2; do
  run gemma3-270m-lora MFT_CE_BUDGET_GB=32
  run gemma3-270m-lora MFT_CE_BUDGET_GB=4
  run gemma3-270m-lora MFT_CE_BUDGET_GB=2
  run gemma3-270m-lora MFT_CE_BUDGET_GB=4 MFT_GEMM8_STREAM=5
  run gpt2-lora MFT_CE_BUDGET_GB=32
  run gpt2-lora MFT_CE_BUDGET_GB=4
  run gpt2-lora MFT_CE_BUDGET_GB=32 MFT_GEMM8_STREAM=5
  run gpt2-lora MFT_CE_BUDGET_GB=32 MFT_GEMM8_ALL=1
  run gemma3-270m-lora MFT_CE_BUDGET_GB=4 MFT_GEMM8_ALL=1
done
