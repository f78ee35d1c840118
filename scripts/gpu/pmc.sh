#!/bin/bash
# One rocprofv3 PMC pass (its own run: never combined with tracing domains) over a command, summarised per
# kernel by scripts/pmc_db.py.  Counter budget per pass on gfx950: 8 SQ, 4 TCC (FETCH_SIZE = 3, WRITE_SIZE
# = 2), 4 TCP, 2 TA, 2 TD, 2 GRBM -- more prints "error code 38" and hangs, hence the hard KILL timeout.
#   scripts/gpu/pmc.sh <tag> "<counters>" <program> [args...]
#   e.g. scripts/gpu/pmc.sh attn256 "SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_INSTS_MFMA" \
#            python3 scripts/bench_attn256.py
set -o pipefail
TAG=$1; CNT=$2; shift 2
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/pmc_$TAG
mkdir -p $O && cd /tmp && export TMPDIR=/tmp PYTHONPATH=$R
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $CNT -d $O -o run -- "$@" > $O/run.log 2>&1 || { tail -20 $O/run.log; exit 1; }
python3 $R/scripts/pmc_db.py $(find $O -name "*.db" | head -1) > $R/gpurun_out/${TAG}_pmc.txt 2>&1
rm -rf $O/*/
head -40 $R/gpurun_out/${TAG}_pmc.txt | cut -c1-200
