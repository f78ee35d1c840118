#!/bin/bash
# D = 256 attention forward with swizzled (conflict-free) K / V pair images: numerics, A/B vs the plain
# images (MFT_ATTN_SWZ=0), PMC of both; then the 4 x 128 recipe profiled eagerly, and (last: it may
# crash inside rocprofiler) in graph mode at 16 x 128
set -o pipefail
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "attn or attention" \
  tests/test_engine_gemma_gpu.py > gpurun_out/r4b5_tests.log 2>&1; rc=$?
tail -2 gpurun_out/r4b5_tests.log
[ $rc -eq 0 ] || exit 1
for r in 1 2; do
  for sw in 0 1; do
    MFT_ATTN_SWZ=$sw timeout -k 10 120 python3 scripts/bench_attn256.py 2>&1 | grep -v amdgpu.ids | sed "s/^/swz=$sw /" || exit 1
  done
done | tee gpurun_out/r4b5_attn_ab.txt
for sw in 0 1; do
  MFT_ATTN_SWZ=$sw timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT -d gpurun_out/pmc/s$sw -o run -- python3 scripts/diag/attn256_pmc_probe.py > gpurun_out/pmc/s$sw.log 2>&1 || exit 1
  DB=$(find gpurun_out/pmc/s$sw -name "*.db" | head -1)
  echo "== MFT_ATTN_SWZ=$sw"; python3 scripts/pmc_db.py $DB attn_fwd
  rm -rf gpurun_out/pmc/s$sw
done | tee gpurun_out/r4b5_attn_pmc.txt
A="--random_init --synthetic_data --synthetic_tokens 200000 --seq_len 128 --steps 60 --log_interval 0 --bench_steps 40 --bench_warmup 10"
rm -rf gpurun_out/p_b4
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/p_b4 -o run -- mobilefinetuner_amd/bin/gpt2_lora_finetune $A --batch_size 4 --no_graph > gpurun_out/r4b5_b4_eager_prof.log 2>&1 || { tail -5 gpurun_out/r4b5_b4_eager_prof.log; exit 1; }
grep MFT_BENCH gpurun_out/r4b5_b4_eager_prof.log | cut -c1-120
DB=$(find gpurun_out/p_b4 -name "*.db" | head -1)
python3 scripts/prof_db.py $DB stats 60 40 > gpurun_out/r4b5_b4_eager_kernel_stats.txt && head -20 gpurun_out/r4b5_b4_eager_kernel_stats.txt | cut -c1-150
python3 scripts/prof_db.py $DB step > gpurun_out/r4b5_b4_eager_step.txt 2>&1; tail -1 gpurun_out/r4b5_b4_eager_step.txt
rm -rf gpurun_out/p_b4
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/p_b16 -o run -- mobilefinetuner_amd/bin/gpt2_lora_finetune $A --batch_size 16 > gpurun_out/r4b5_b16_graph_prof.log 2>&1; rc=$?
echo "graph-mode profile at 16 x 128: rc=$rc"; grep -A3 "fatal signal" gpurun_out/r4b5_b16_graph_prof.log | head -4
rm -rf gpurun_out/p_b16
exit 0
