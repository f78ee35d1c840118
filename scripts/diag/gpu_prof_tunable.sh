#!/bin/bash
# kernel stats of the headline bench with the shipped TunableOp database (GEMM kernel shapes)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD

rm -rf gpurun_out/tprof
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/tprof -o run -- python3 bench.py --steps 10 --warmup 3 > gpurun_out/tprof.log 2>&1 || { tail gpurun_out/tprof.log; exit 1; }
DB=$(find gpurun_out/tprof -name "*.db" | head -1)
python3 scripts/prof_db.py $DB stats 13 30 > gpurun_out/tprof_stats.txt && head -22 gpurun_out/tprof_stats.txt
python3 - "$DB" <<'PY'
import sqlite3, sys
c = sqlite3.connect(f"file:{sys.argv[1]}?mode=ro", uri=True)
names = set(r[0] for r in c.execute("select distinct name from kernels") if 'Cijk' in r[0] or 'rocblas' in r[0].lower())
for n in sorted(names): print(n[:250])
PY
rm -rf gpurun_out/tprof
