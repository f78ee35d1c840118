#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 200 python3 scripts/diag/z2_debug.py 2>&1 | grep -v amdgpu.ids | tail -12
