# per-kernel hardware counters of the split attention kernels (one counter pass per run)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 120 python3 $R/scripts/bench_attn.py > $R/gpurun_out/attn_micro.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD -d $R/gpurun_out/pmc_attn1 -o run -- python3 $R/scripts/bench_attn.py --iters 3 > $R/gpurun_out/pmc1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE -d $R/gpurun_out/pmc_attn2 -o run -- python3 $R/scripts/bench_attn.py --iters 3 > $R/gpurun_out/pmc2.log 2>&1 || exit 1
