#!/bin/bash
# dQ kernel on swizzled K/V images; the two-rank GEMM choice map test; Gemma bench; then (last: may crash
# inside rocprofiler) graph-mode profiling at 16 x 128 with no hipBLASLt kernel in the graph
set -o pipefail
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "attn or attention" \
  tests/test_engine_gemma_gpu.py "tests/test_engine_dist_gpu.py::test_native_two_ranks_print_identical_gemm_choice_maps" \
  "tests/test_engine_dist_gpu.py::test_native_dp_lora_and_gemma_two_ranks" > gpurun_out/r4b6_tests.log 2>&1; rc=$?
tail -2 gpurun_out/r4b6_tests.log
[ $rc -eq 0 ] || { grep -B5 -A30 "Error\|FAIL" gpurun_out/r4b6_tests.log | head -60; exit 1; }
for r in 1 2; do timeout -k 10 120 python3 scripts/bench_attn256.py 2>&1 | grep -v amdgpu.ids || exit 1; done | tee gpurun_out/r4b6_attn.txt
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT -d gpurun_out/pmc/q -o run -- python3 scripts/diag/attn256_pmc_probe.py > gpurun_out/pmc/q.log 2>&1 || exit 1
DB=$(find gpurun_out/pmc/q -name "*.db" | head -1); python3 scripts/pmc_db.py $DB attn_ | tee gpurun_out/r4b6_attn_pmc.txt; rm -rf gpurun_out/pmc/q
timeout -k 10 300 python3 bench.py --config gemma3-270m-lora --steps 20 --warmup 5 > gpurun_out/r4b6_bench_gemma.txt 2>&1 || { tail -5 gpurun_out/r4b6_bench_gemma.txt; exit 1; }
tail -1 gpurun_out/r4b6_bench_gemma.txt | cut -c1-200
A="--random_init --synthetic_data --synthetic_tokens 200000 --seq_len 128 --steps 60 --log_interval 0 --bench_steps 40 --bench_warmup 10"
MFT_GEMM8_ALL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/p_b16 -o run -- mobilefinetuner_amd/bin/gpt2_lora_finetune $A --batch_size 16 > gpurun_out/r4b6_b16_graph_prof.log 2>&1; rc=$?
echo "graph-mode profile at 16 x 128, MFT_GEMM8_ALL=1: rc=$rc"; grep -A3 "fatal signal" gpurun_out/r4b6_b16_graph_prof.log | head -4
if [ $rc -eq 0 ]; then DB=$(find gpurun_out/p_b16 -name "*.db" | head -1); python3 scripts/prof_db.py $DB stats 60 30 > gpurun_out/r4b6_b16_graph_kernel_stats.txt; head -5 gpurun_out/r4b6_b16_graph_kernel_stats.txt | cut -c1-120; fi
rm -rf gpurun_out/p_b16
exit 0
