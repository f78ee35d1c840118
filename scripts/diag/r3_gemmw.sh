#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 400 python3 -u scripts/bench_gemmw.py --rounds 3 > gpurun_out/r3_gemmw_bench.txt 2>&1 || { tail -30 gpurun_out/r3_gemmw_bench.txt; exit 1; }
cat gpurun_out/r3_gemmw_bench.txt
