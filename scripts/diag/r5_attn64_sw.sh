#!/bin/bash
# swizzled short-path attention images: attention tests, timing, LDS conflict counters, headline bench
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5a64sw
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$R
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "attention or attn" > $O/tests.txt 2>&1; rc=$?; tail -2 $O/tests.txt; [ $rc -eq 0 ] || { grep -B3 -A30 "Error\|FAIL" $O/tests.txt | head -60; exit 1; }
timeout -k 10 120 python3 scripts/diag/attn64_pmc_probe.py 20 > $O/time.txt 2>&1 || { tail -5 $O/time.txt; exit 1; }
cat $O/time.txt
cd /tmp
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT -d $O/p1 -o run -- python3 $R/scripts/diag/attn64_pmc_probe.py 3 > $O/p1.log 2>&1 || { tail -5 $O/p1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_MFMA -d $O/p2 -o run -- python3 $R/scripts/diag/attn64_pmc_probe.py 3 > $O/p2.log 2>&1 || { tail -5 $O/p2.log; exit 1; }
cd $R
for p in p1 p2; do python3 scripts/pmc_db.py $(find $O/$p -name "*.db" | head -1) attn > $O/$p.txt 2>&1; cat $O/$p.txt | head -24; done
rm -rf $O/p1 $O/p2
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --config gpt2-lora --steps 20 --warmup 5 > $O/one.txt 2>&1 || { tail -5 $O/one.txt; exit 1; }
  echo "headline $(tail -1 $O/one.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), d["ms_per_step"])')"
done
