#!/bin/bash
# store-pattern probe + native DP / ZeRO tests (replicated fp32 bucket, export gather, update-delta check)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/diag/r4_store_probe.hip -o /tmp/r4_store_probe 2>/dev/null || exit 1
timeout -k 10 120 /tmp/r4_store_probe > gpurun_out/r4_store_probe2.txt 2>&1 || { cat gpurun_out/r4_store_probe2.txt; exit 1; }
cat gpurun_out/r4_store_probe2.txt
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_engine_dist_gpu.py tests/test_engine_gemma_gpu.py -k "two_ranks_match or lora_and_gemma or peer_failure or rccl or embedding_dump" > gpurun_out/r4_dist_tests.log 2>&1; rc=$?
tail -25 gpurun_out/r4_dist_tests.log
exit $rc
