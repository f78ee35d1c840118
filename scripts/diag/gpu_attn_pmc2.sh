# split attention after the LDS pitch change: tests, micro-bench, one counter pass, Gemma bench
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "attention" > gpurun_out/t_attn4.log 2>&1 || exit 1
timeout -k 10 120 python3 scripts/bench_attn.py > gpurun_out/attn_micro2.log 2>&1 || exit 1
timeout -k 10 180 python bench.py --config gemma3-270m-lora --steps 15 --warmup 4 > gpurun_out/b_attn4.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE -d $R/gpurun_out/pmc_attn3 -o run -- python3 $R/scripts/bench_attn.py --iters 3 > $R/gpurun_out/pmc3.log 2>&1 || exit 1
