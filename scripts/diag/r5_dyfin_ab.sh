#!/bin/bash
# lora_dy in-kernel finish (default) vs separate finish kernel (MFT_LORA_DY_FIN=0), interleaved on one box
set -o pipefail
O=gpurun_out/r5dyfinab
mkdir -p $O
for r in 1 2; do
  for f in 1 0; do
    for c in gpt2-lora gemma3-270m-lora; do
      MFT_LORA_DY_FIN=$f timeout -k 10 300 python3 bench.py --config $c --steps 20 --warmup 5 > $O/one.txt 2>&1 || { tail -5 $O/one.txt; exit 1; }
      echo "round $r fin=$f $c $(tail -1 $O/one.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), d["ms_per_step"])')"
    done
  done
done
