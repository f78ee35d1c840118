#!/bin/bash
# MFT_GEMM8_ALL A/B: plain NT forwards on gemm8 (1) vs tuned hipBLASLt (0)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py > gpurun_out/g8all_tests.log 2>&1 || { tail -30 gpurun_out/g8all_tests.log; exit 1; }
tail -1 gpurun_out/g8all_tests.log
: > gpurun_out/g8all_ab.txt
for c in gemma3-270m-lora gpt2-lora; do
  for r in 1 2; do
    for v in 0 1; do
      out=$(MFT_GEMM8_ALL=$v timeout -k 10 300 python3 bench.py --config $c --steps 20 --warmup 5 2> gpurun_out/g8all_ab.err) || { tail -5 gpurun_out/g8all_ab.err; exit 1; }
      echo "$c g8all=$v $(echo "$out" | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')" | tee -a gpurun_out/g8all_ab.txt
    done
  done
done
prof() {  # tag, steps, bench args...
  local tag=$1 n=$2; shift 2
  rm -rf gpurun_out/p_$tag
  timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/p_$tag -o run -- python3 bench.py --steps $n --warmup 3 "$@" > gpurun_out/p_$tag.log 2>&1 || { tail gpurun_out/p_$tag.log; return 1; }
  DB=$(find gpurun_out/p_$tag -name "*.db" | head -1)
  python3 scripts/prof_db.py $DB stats $((n + 3)) 40 > gpurun_out/${tag}_stats.txt && grep -i "gemm8\|cijk\|total" gpurun_out/${tag}_stats.txt | cut -c1-150
  rm -rf gpurun_out/p_$tag
}
MFT_GEMM8_ALL=1 prof gemma_g8all 6 --config gemma3-270m-lora
