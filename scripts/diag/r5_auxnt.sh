#!/bin/bash
# gemm4 epilogue aux loads: non-temporal (default) vs default policy; epilogue kernels, then the headline, interleaved
set -o pipefail
O=gpurun_out/r5auxnt
mkdir -p $O
export PYTHONPATH=.
for p in nt plain nt plain; do
  MFT_G4_AUX=$p timeout -k 10 300 python3 scripts/bench_gemm4.py --epi --shapes "gpt2 fc fwd,gpt2 proj fwd" > $O/e_$p.txt 2>&1 || { tail -5 $O/e_$p.txt; exit 1; }
  echo "aux=$p"; grep "|" $O/e_$p.txt | cut -c1-170
done
for r in 1 2; do
  for p in nt plain; do
    MFT_G4_AUX=$p timeout -k 10 300 python3 bench.py --config gpt2-lora --steps 20 --warmup 5 > $O/one.txt 2>&1 || { tail -5 $O/one.txt; exit 1; }
    echo "round $r aux $p $(tail -1 $O/one.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), d["ms_per_step"])')"
  done
done
