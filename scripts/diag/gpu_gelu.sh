#!/bin/bash
# GELU' stored in the fc epilogue: gemm / model / engine GPU tests, headline bench + kernel stats
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py tests/test_models_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/gelu_tests.log 2>&1 || { tail -30 gpurun_out/gelu_tests.log; exit 1; }
tail -2 gpurun_out/gelu_tests.log
: > gpurun_out/gelu_bench.jsonl
for c in gpt2-lora gpt2-full; do
timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 >> gpurun_out/gelu_bench.jsonl 2>gpurun_out/gelu_bench.err || { tail gpurun_out/gelu_bench.err; exit 1; }
done
cut -c1-260 gpurun_out/gelu_bench.jsonl
rm -rf gpurun_out/pg
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/pg -o run -- python3 bench.py --steps 10 --warmup 3 > gpurun_out/pg.log 2>&1 || { tail gpurun_out/pg.log; exit 1; }
DB=$(find gpurun_out/pg -name "*.db" | head -1)
python3 scripts/prof_db.py $DB stats 13 30 > gpurun_out/gpt2_gelu_stats.txt && head -12 gpurun_out/gpt2_gelu_stats.txt
rm -rf gpurun_out/pg
