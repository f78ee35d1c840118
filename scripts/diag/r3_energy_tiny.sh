#!/bin/bash
# bench energy reporting (rank-0 GPU power over the timed steps) + tiny-model bf16-vs-fp32 errors
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r3_energy.json 2> gpurun_out/r3_energy.err || { tail -20 gpurun_out/r3_energy.err; exit 1; }
python3 -c 'import json; r=json.load(open("gpurun_out/r3_energy.json")); print(r["value"], r["config"]["gpu_energy_rank0"])'
timeout -k 10 300 python3 scripts/diag/tiny_parity_errors.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r3_tiny_errors.txt
