#!/bin/bash
set -o pipefail
O=gpurun_out/${1:-r5m}
mkdir -p $O
timeout -k 10 300 python3 scripts/bench_gemm4.py --epi --shapes "gpt2 fc fwd,gpt2 proj fwd,gpt2 qkv fwd (aug K),gemma gate|up fwd,gemma down fwd" > $O/epi.txt 2>&1 || { tail -20 $O/epi.txt; exit 1; }
timeout -k 10 300 python3 scripts/bench_gemm4.py --rounds 5 > $O/all.txt 2>&1 || { tail -20 $O/all.txt; exit 1; }
cat $O/*.txt | grep -v amdgpu.ids
