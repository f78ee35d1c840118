#!/bin/bash
# gemm4: BIAS_ADD epilogue check + store cache policy A/B (MFT_G4_PDIAG=3: non-temporal epilogue stores)
set -o pipefail
O=gpurun_out/${1:-r5l}
mkdir -p $O
SH="gpt2 fc fwd,gpt2 proj fwd,gpt2 qkv fwd (aug K),gpt2 lm head,8192^3"
timeout -k 10 200 python3 scripts/bench_gemm4.py --epi --shapes "gpt2 fc fwd,gpt2 proj fwd" > $O/epi.txt 2>&1 || { tail -20 $O/epi.txt; exit 1; }
timeout -k 10 200 python3 scripts/bench_gemm4.py --shapes "$SH" --rounds 5 > $O/pol0.txt 2>&1 || { tail -20 $O/pol0.txt; exit 1; }
MFT_G4_PDIAG=3 timeout -k 10 200 python3 scripts/bench_gemm4.py --shapes "$SH" --rounds 5 > $O/pol3.txt 2>&1 || { tail -20 $O/pol3.txt; exit 1; }
cat $O/*.txt | grep -v amdgpu.ids
