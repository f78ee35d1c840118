#!/bin/bash
# kernel stats of the headline step at the default micro-batch (rocprofv3 --kernel-trace)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
rm -rf gpurun_out/p_head
timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/p_head -o run -- python3 bench.py --steps 8 --warmup 3 > gpurun_out/p_head.log 2>&1 || { tail gpurun_out/p_head.log; exit 1; }
DB=$(find gpurun_out/p_head -name "*.db" | head -1)
python3 scripts/prof_db.py $DB stats 11 40 > gpurun_out/head_stats.txt && head -22 gpurun_out/head_stats.txt | cut -c1-150
rm -rf gpurun_out/p_head
tail -1 gpurun_out/p_head.log | cut -c1-200
