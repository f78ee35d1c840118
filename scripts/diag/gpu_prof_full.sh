#!/bin/bash
# kernel stats of the gpt2-full bench step
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
rm -rf gpurun_out/p_full
timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/p_full -o run -- python3 bench.py --config gpt2-full --steps 8 --warmup 3 > gpurun_out/p_full.log 2>&1 || { tail gpurun_out/p_full.log; exit 1; }
DB=$(find gpurun_out/p_full -name "*.db" | head -1)
python3 scripts/prof_db.py $DB stats 11 40 > gpurun_out/full_stats.txt && head -30 gpurun_out/full_stats.txt | cut -c1-160
rm -rf gpurun_out/p_full
