#!/bin/bash
# staged host-moment ZeRO-3 optimizer in eager mode (its stream pattern crashes hipStreamEndCapture) vs in place
set -o pipefail
O=gpurun_out/${1:-r5staged2}
mkdir -p $O
for v in "0 - graph" "1 - eager" "0 - eager" "1 12 eager" "1 49 eager"; do
  set -- $v
  G=""; [ "$3" = eager ] && G="--no-graph"
  S=""; [ "$2" != "-" ] && S="$2"
  MFT_Z3_STAGED=$1 MFT_Z3_SLOTS=$S timeout -k 10 400 python3 bench.py --config gpt2-xl-zero3-offload --steps 10 --warmup 3 $G > $O/b.txt 2>&1 || { tail -5 $O/b.txt; exit 1; }
  echo "staged=$1 slots=$2 $3: $(tail -1 $O/b.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), "tok/s", d["ms_per_step"], "ms/step", d["config"].get("peak_hbm_gb_rank0"), "GB")')"
done
