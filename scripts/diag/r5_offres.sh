#!/bin/bash
# ZeRO-3 + host AdamW (gpt2-xl): gemm4 grids leaving the streamed updates' CUs free, on / off
set -o pipefail
O=gpurun_out/${1:-r5offres}
mkdir -p $O
for r in 0 1 0 1; do
  MFT_Z3_RESERVE=$r timeout -k 10 400 python3 bench.py --config gpt2-xl-zero3-offload --steps 10 --warmup 3 > $O/b_$r.txt 2>&1 || { tail -5 $O/b_$r.txt; exit 1; }
  echo "reserve=$r: $(tail -1 $O/b_$r.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), "tok/s", d["ms_per_step"], "ms/step")')"
done
