#!/bin/bash
# D=256 dQ variants: DMA ring slots (2/3) x delta folded into dQ (1/0); per-kernel times
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 400 python3 -u -m pytest tests/test_kernels_gpu.py -k "attention" -q --timeout 300 --timeout-method thread \
  > gpurun_out/r3_attndq_tests.log 2>&1; rc=$?; echo "attention tests rc=$rc"; grep -E "passed|failed" gpurun_out/r3_attndq_tests.log | tail -2
[ $rc -eq 0 ] || exit 1
for ring in 2 3; do for fold in 1 0; do
  rm -rf gpurun_out/p_attn
  MFT_ATTN_DQ_RING=$ring MFT_ATTN_DELTA_FOLD=$fold timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/p_attn -o run -- python3 scripts/bench_attn256.py > gpurun_out/r3_attn_prof.log 2>&1 || { tail gpurun_out/r3_attn_prof.log; exit 1; }
  DB=$(find gpurun_out/p_attn -name "*.db" | head -1)
  echo "== ring=$ring fold=$fold"; python3 scripts/prof_db.py $DB stats 1 5 | grep -E "attn" | cut -c1-110
done; done
rm -rf gpurun_out/p_attn
