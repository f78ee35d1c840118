#!/bin/bash
# GPU-side kernel times of the short-token GEMMs (gemm4 / gemm_s / hipBLASLt) at the 4 x 128 recipe shapes
set -o pipefail
O=gpurun_out/${1:-r5gs}
mkdir -p $O
export TMPDIR=/tmp
rm -rf $O/p
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p -o run -- python3 scripts/bench_gemm4.py --shapes "${SH:-b4 proj fwd,b4 fc fwd,b4 mproj fwd}" --rounds 3 --iters 20 --only gemm4,gemm_s,hipBLASLt > $O/log.txt 2>&1 || { tail -5 $O/log.txt; exit 1; }
python3 scripts/prof_db.py $(find $O/p -name "*.db" | head -1) stats 1 30 > $O/stats.txt && head -30 $O/stats.txt | cut -c1-170
rm -rf $O/p
