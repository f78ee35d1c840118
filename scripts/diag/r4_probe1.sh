#!/bin/bash
# round 4 first probe: per-CU store / fill rates (lockstep vs sparse grids), gemm8 tile-phase stamps,
# headline bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/diag/r4_store_probe.hip -o /tmp/r4_store_probe 2>/dev/null || exit 1
hipcc --offload-arch=gfx950 -O3 -std=c++17 -DMFT_G8_STAMPS -I mobilefinetuner_amd/csrc scripts/diag/g8_stamps.hip -o /tmp/g8_stamps 2>/dev/null || exit 1
timeout -k 10 120 /tmp/r4_store_probe > gpurun_out/r4_store_probe.txt 2>&1 || { cat gpurun_out/r4_store_probe.txt; exit 1; }
cat gpurun_out/r4_store_probe.txt
timeout -k 10 120 /tmp/g8_stamps > gpurun_out/r4_g8_stamps.txt 2>&1 || { cat gpurun_out/r4_g8_stamps.txt; exit 1; }
cat gpurun_out/r4_g8_stamps.txt
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r4_bench0.txt 2>&1 || { tail -20 gpurun_out/r4_bench0.txt; exit 1; }
tail -2 gpurun_out/r4_bench0.txt
