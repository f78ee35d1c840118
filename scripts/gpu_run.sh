#!/bin/bash
# Development GPU check: gpu tests, bench (headline + optional extra configs), rocprofv3 kernel stats
# of the headline step.  usage: bash scripts/gpu_run.sh [tag] [extra bench configs...]
set -o pipefail
TAG=${1:-dev}; shift
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -4 gpurun_out/${TAG}_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python bench.py --steps 30 --warmup 5 > gpurun_out/${TAG}_bench.jsonl 2> gpurun_out/${TAG}_bench.err || { tail gpurun_out/${TAG}_bench.err; exit 1; }
for c in "$@"; do
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 >> gpurun_out/${TAG}_bench.jsonl 2>> gpurun_out/${TAG}_bench.err || { tail gpurun_out/${TAG}_bench.err; exit 1; }
done
cat gpurun_out/${TAG}_bench.jsonl
rm -rf gpurun_out/${TAG}_prof
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/${TAG}_prof -o run -- python3 bench.py --steps 10 --warmup 3 > gpurun_out/${TAG}_prof.log 2>&1 || { tail gpurun_out/${TAG}_prof.log; exit 1; }
DB=$(find gpurun_out/${TAG}_prof -name "*.db" | head -1)
python3 scripts/prof_db.py $DB stats 13 30 > gpurun_out/${TAG}_kernel_stats.txt && head -25 gpurun_out/${TAG}_kernel_stats.txt
rm -rf gpurun_out/${TAG}_prof
