#!/bin/bash
# round-2 closing run (rebuilt tree): full GPU suite, smoke, every bench config, LoRA kernel stats
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/final2_gpu_tests.log 2>&1 || { tail -30 gpurun_out/final2_gpu_tests.log; exit 1; }
tail -1 gpurun_out/final2_gpu_tests.log
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final2_smoke.log 2>&1 || { tail -20 gpurun_out/final2_smoke.log; exit 1; }
echo smoke ok
: > gpurun_out/final2_bench.jsonl
for c in gpt2-lora gemma3-270m-lora gpt2-full gpt2-xl-zero gpt2-xl-zero3 gpt2-xl-zero3-offload; do
  timeout -k 10 400 python3 bench.py --config $c --steps 20 --warmup 5 >> gpurun_out/final2_bench.jsonl 2> gpurun_out/final2_$c.err || { tail -5 gpurun_out/final2_$c.err; exit 1; }
  tail -1 gpurun_out/final2_bench.jsonl | cut -c1-200
done
prof() {  # tag, steps, bench args...
  local tag=$1 n=$2; shift 2
  rm -rf gpurun_out/p_$tag
  timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/p_$tag -o run -- python3 bench.py --steps $n --warmup 3 "$@" > gpurun_out/p_$tag.log 2>&1 || { tail gpurun_out/p_$tag.log; return 1; }
  DB=$(find gpurun_out/p_$tag -name "*.db" | head -1)
  python3 scripts/prof_db.py $DB stats $((n + 3)) 40 > gpurun_out/${tag}_stats.txt && head -4 gpurun_out/${tag}_stats.txt | cut -c1-150
  rm -rf gpurun_out/p_$tag
}
prof final2_gpt2 10 && prof final2_gemma 6 --config gemma3-270m-lora
