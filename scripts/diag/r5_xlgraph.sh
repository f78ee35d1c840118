#!/bin/bash
# gpt2-xl ZeRO-2 / ZeRO-3: hipGraph step vs eager
set -o pipefail
O=gpurun_out/${1:-r5xlg}
mkdir -p $O
for v in "gpt2-xl-zero3 graph" "gpt2-xl-zero3 eager" "gpt2-xl-zero graph" "gpt2-xl-zero eager"; do
  set -- $v
  G=""; [ "$2" = eager ] && G="--no-graph"
  timeout -k 10 400 python3 bench.py --config $1 --steps 10 --warmup 3 $G > $O/b.txt 2>&1 || { tail -5 $O/b.txt; exit 1; }
  echo "$1 $2: $(tail -1 $O/b.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), "tok/s", d["ms_per_step"], "ms/step", d["config"].get("peak_hbm_gb_rank0"), "GB")')"
done
