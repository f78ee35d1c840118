#!/bin/bash
# gemm8 N-tail quadrant skip: GEMM + LM-head CE tests, LoRA benches, Gemma kernel stats
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py tests/test_lm_head_ce_gpu.py > gpurun_out/ntail_tests.log 2>&1 || { tail -30 gpurun_out/ntail_tests.log; exit 1; }
tail -1 gpurun_out/ntail_tests.log
: > gpurun_out/ntail_bench.jsonl
for c in gemma3-270m-lora gpt2-lora; do
  timeout -k 10 400 python3 bench.py --config $c --steps 20 --warmup 5 >> gpurun_out/ntail_bench.jsonl 2> gpurun_out/ntail_$c.err || { tail -5 gpurun_out/ntail_$c.err; exit 1; }
  tail -1 gpurun_out/ntail_bench.jsonl | cut -c1-200
done
prof() {  # tag, steps, bench args...
  local tag=$1 n=$2; shift 2
  rm -rf gpurun_out/p_$tag
  timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/p_$tag -o run -- python3 bench.py --steps $n --warmup 3 "$@" > gpurun_out/p_$tag.log 2>&1 || { tail gpurun_out/p_$tag.log; return 1; }
  DB=$(find gpurun_out/p_$tag -name "*.db" | head -1)
  python3 scripts/prof_db.py $DB stats $((n + 3)) 40 > gpurun_out/${tag}_stats.txt && head -12 gpurun_out/${tag}_stats.txt | cut -c1-150
  rm -rf gpurun_out/p_$tag
}
prof gemma_ntail 6 --config gemma3-270m-lora
