#!/bin/bash
# Closing run of a tree: the GPU test tier (as the driver runs it), the smoke step, then every bench config.
#   scripts/gpu/close.sh <tag>   -> gpurun_out/<tag>_tests.log, <tag>_bench.jsonl
set -o pipefail
TAG=$1
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R
timeout -k 10 1500 python3 -u -m pytest tests -m gpu -x -v --timeout 170 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 \
  || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -3 gpurun_out/${TAG}_tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail gpurun_out/${TAG}_smoke.log; exit 1; }
: > gpurun_out/${TAG}_bench.jsonl
for c in gpt2-lora gemma3-270m-lora gemma3-1b-lora gpt2-full gpt2-xl-zero gpt2-xl-zero3 gpt2-xl-zero3-offload; do
  timeout -k 10 400 python3 bench.py --config $c --steps 20 --warmup 5 >> gpurun_out/${TAG}_bench.jsonl 2>gpurun_out/${TAG}_bench_$c.err \
    || { echo "bench $c failed"; tail gpurun_out/${TAG}_bench_$c.err; exit 1; }
done
timeout -k 10 200 python3 bench.py --batch 4 --steps 50 --warmup 10 >> gpurun_out/${TAG}_bench.jsonl 2>/dev/null || exit 1
cut -c1-160 gpurun_out/${TAG}_bench.jsonl
