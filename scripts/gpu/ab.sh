#!/bin/bash
# Interleaved A/B of environment settings on one bench.py configuration (boxes differ by a few percent:
# compare arms on the same box, rounds interleaved).
#   scripts/gpu/ab.sh <tag> <rounds> "<env A>" "<env B>" [bench.py args...]
#   e.g. scripts/gpu/ab.sh g4aux 3 "MFT_G4_AUX=nt" "MFT_G4_AUX=plain" --config gpt2-lora --steps 20
# -> gpurun_out/<tag>_ab.jsonl (one line per run, "arm" added)
set -o pipefail
TAG=$1; N=$2; A=$3; B=$4; shift 4
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out/${TAG}_ab.jsonl
: > $OUT
for i in $(seq 1 $N); do
  for arm in A B; do
    ENVS=$A; [ $arm = B ] && ENVS=$B
    L=$(env $ENVS timeout -k 10 400 python3 $R/bench.py "$@" 2>/dev/null | tail -1) || { echo "arm $arm failed"; exit 1; }
    echo "$L" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); d['arm']='$arm: $ENVS'; print(json.dumps(d))" >> $OUT
    echo "$arm ($ENVS): $(echo "$L" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
  done
done
