#!/bin/bash
# gemm8 (8-phase) vs the 4-phase form (32-MFMA segments) vs hipBLASLt on the NT training shapes
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 400 python3 scripts/bench_g8late.py --variants 0,4 --rounds 4 > gpurun_out/r4_p2.txt 2>&1 || { tail -30 gpurun_out/r4_p2.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r4_p2.txt
