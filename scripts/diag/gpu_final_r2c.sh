#!/bin/bash
# round-2 final tree: full GPU suite, smoke, headline + Gemma bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/final3_gpu_tests.log 2>&1 || { tail -30 gpurun_out/final3_gpu_tests.log; exit 1; }
tail -1 gpurun_out/final3_gpu_tests.log
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final3_smoke.log 2>&1 || { tail -20 gpurun_out/final3_smoke.log; exit 1; }
echo smoke ok
: > gpurun_out/final3_bench.jsonl
for c in gpt2-lora gemma3-270m-lora; do
  timeout -k 10 400 python3 bench.py --config $c --steps 20 --warmup 5 >> gpurun_out/final3_bench.jsonl 2> gpurun_out/final3_$c.err || { tail -5 gpurun_out/final3_$c.err; exit 1; }
  tail -1 gpurun_out/final3_bench.jsonl | cut -c1-200
done
timeout -k 10 300 python3 bench.py > gpurun_out/final3_default.json 2> gpurun_out/final3_default.err || { tail -5 gpurun_out/final3_default.err; exit 1; }
cat gpurun_out/final3_default.json
