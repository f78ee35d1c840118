#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
MFT_TEST_GRAPH_COMM=1 timeout -k 10 400 python3 -u -m pytest tests/test_dp_graph_gpu.py -v --timeout 240 \
  --timeout-method thread > gpurun_out/r3_avgfix_py.log 2>&1; echo "python dp graph rc=$?"; grep -E "PASSED|FAILED|Error" gpurun_out/r3_avgfix_py.log | tail -10
timeout -k 10 900 python3 -u -m pytest tests/test_engine_dist_gpu.py -x -q --timeout 240 --timeout-method thread > gpurun_out/r3_avgfix_nat.log 2>&1; echo "native dist rc=$?"; tail -3 gpurun_out/r3_avgfix_nat.log
