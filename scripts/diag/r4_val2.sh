#!/bin/bash
# the two re-fixed tests, then the benches of r4_val.sh
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 400 python -u -m pytest -v --timeout 300 --timeout-method thread \
  tests/test_kernels_gpu.py::test_adamw_amsgrad_matches_torch \
  tests/test_engine_gemma_gpu.py::test_native_gemma_embedding_dump_and_token_preview > gpurun_out/r4_val2_tests.log 2>&1; rc=$?
tail -4 gpurun_out/r4_val2_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
bash scripts/diag/r4_val.sh bench
