#!/bin/bash
# round-3 closing run, part 1: every GPU test + the smoke step on this tree
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r3_final_gpu_tests.log 2>&1; echo "gpu tests rc=$?"
grep -E "passed|failed" gpurun_out/r3_final_gpu_tests.log | tail -3
grep -E "^FAILED" gpurun_out/r3_final_gpu_tests.log | head -20
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3_final_smoke.log 2>&1; echo "smoke rc=$?"; tail -3 gpurun_out/r3_final_smoke.log
