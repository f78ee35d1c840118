#!/bin/bash
set -o pipefail
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 200 python3 scripts/diag/z2_debug.py 2>&1 | grep -v amdgpu.ids | grep -E "mismatch|rel diff|sync" | tail -8
