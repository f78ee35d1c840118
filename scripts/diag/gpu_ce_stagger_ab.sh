#!/bin/bash
# CE forward workgroup stagger A/B (MFT_CE_STAGGER = s_sleep(127) count for half of the CUs; 0 = off)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_lm_head_ce_gpu.py > gpurun_out/stagger_tests.log 2>&1 || { tail -30 gpurun_out/stagger_tests.log; exit 1; }
tail -1 gpurun_out/stagger_tests.log
: > gpurun_out/stagger_ab.txt
for c in gpt2-lora gemma3-270m-lora; do
  for r in 1 2; do
    for v in 0 2 4 6; do
      out=$(MFT_CE_STAGGER=$v timeout -k 10 300 python3 bench.py --config $c --steps 20 --warmup 5 2> gpurun_out/stagger_ab.err) || { tail -5 gpurun_out/stagger_ab.err; exit 1; }
      echo "$c stagger=$v $(echo "$out" | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')" | tee -a gpurun_out/stagger_ab.txt
    done
  done
done
