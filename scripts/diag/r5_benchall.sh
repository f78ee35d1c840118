#!/bin/bash
# every bench config once (plus the headline twice and the reference recipe), JSON lines -> gpurun_out/$1.jsonl
set -o pipefail
O=gpurun_out/${1:-r5_bench}
: > $O.jsonl
for spec in "${@:2}"; do
  IFS=: read -r cfg extra <<< "$spec"
  timeout -k 10 400 python3 bench.py --config $cfg --steps 20 --warmup 5 $extra > $O.one 2>&1 || { tail -5 $O.one; exit 1; }
  tail -1 $O.one >> $O.jsonl
  echo "$cfg $extra: $(tail -1 $O.one | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), d["ms_per_step"], d["config"].get("peak_hbm_gb_rank0"), d.get("mfu"))')"
done
