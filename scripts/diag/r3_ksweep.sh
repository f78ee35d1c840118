#!/bin/bash
# gemm8 vs hipBLASLt K sweep: main-loop cost per K-tile vs per-tile overhead
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 300 python3 scripts/bench_gemm_ksweep.py > gpurun_out/r3_ksweep.txt 2>&1 || { tail -20 gpurun_out/r3_ksweep.txt; exit 1; }
timeout -k 10 300 python3 scripts/bench_gemm_ksweep.py --M 32768 --N 768 --Ks 768,1536,3072,6144,12288 >> gpurun_out/r3_ksweep.txt 2>&1 || { tail -20 gpurun_out/r3_ksweep.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r3_ksweep.txt
