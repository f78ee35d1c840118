#!/bin/bash
# the driver's GPU tier + smoke on the current tree
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5_gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r5_gpu_tests.log
[ $rc -eq 0 ] || { grep -B5 -A40 "Error\|FAIL" gpurun_out/r5_gpu_tests.log | head -80; exit 1; }
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5_smoke.log 2>&1 || { tail -20 gpurun_out/r5_smoke.log; exit 1; }
tail -2 gpurun_out/r5_smoke.log | cut -c1-200
