#!/bin/bash
# staged host-moment ZeRO-3 optimizer: the ZeRO-3 / offload tests, then the offload bench (eager by construction)
set -o pipefail
O=gpurun_out/${1:-r5staged}
mkdir -p $O
export PYTHONPATH=. TMPDIR=/tmp
timeout -k 10 700 python3 -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_engine_dist_gpu.py -k "zero3 or resume" > $O/tests.txt 2>&1; rc=$?; tail -2 $O/tests.txt; [ $rc -eq 0 ] || { grep -B3 -A40 "Error\|FAIL\|assert" $O/tests.txt | head -80; exit 1; }
for v in "1 -" "1 49" "0 -"; do
  set -- $v
  S=""; [ "$2" != "-" ] && S="$2"
  MFT_Z3_STAGED=$1 MFT_Z3_SLOTS=$S timeout -k 10 400 python3 bench.py --config gpt2-xl-zero3-offload --steps 10 --warmup 3 > $O/b.txt 2>&1 || { tail -5 $O/b.txt; exit 1; }
  echo "staged=$1 slots=$2: $(tail -1 $O/b.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), "tok/s", d["ms_per_step"], "ms/step", d["config"].get("peak_hbm_gb_rank0"), "GB")')"
done
