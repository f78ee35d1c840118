#!/bin/bash
# Kernel table of one bench.py configuration (rocprofv3 --kernel-trace --stats, hipGraph replay unless the
# config runs eagerly), summarised per step by scripts/prof_db.py.
#   scripts/gpu/profile.sh <tag> <steps> [bench.py args...]
#   e.g. scripts/gpu/profile.sh r6_gpt2_lora 10 --config gpt2-lora
# -> gpurun_out/<tag>_kernel_stats.txt (copy the ones worth keeping into profiles/)
set -o pipefail
TAG=$1; STEPS=$2; shift 2
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/prof_$TAG
mkdir -p $O && cd /tmp && export TMPDIR=/tmp PYTHONPATH=$R
timeout -k 10 600 rocprofv3 --kernel-trace -d $O -o run -- python3 $R/bench.py --steps $STEPS --warmup 3 "$@" \
  > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
DB=$(find $O -name "*.db" | head -1)
# warm-up steps run too: the table divides by steps + warmup (every step has the same kernels)
python3 $R/scripts/prof_db.py $DB stats $((STEPS + 3)) 45 > $R/gpurun_out/${TAG}_kernel_stats.txt
rm -rf $O/*/ $DB
head -30 $R/gpurun_out/${TAG}_kernel_stats.txt | cut -c1-160
tail -1 $O/bench.log | cut -c1-300
