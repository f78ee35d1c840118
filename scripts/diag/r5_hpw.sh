#!/bin/bash
set -o pipefail
export PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "attention or attn or flash" 2>&1 | tail -1 || exit 1
for r in 1 2; do for m in 1 2 4; do
  MFT_ATTN_HPW=$m timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/hpw.txt 2>&1 || { tail -5 gpurun_out/hpw.txt; exit 1; }
  echo "hpw=$m $(tail -1 gpurun_out/hpw.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), d["ms_per_step"])')"
done; done
