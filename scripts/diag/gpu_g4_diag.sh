#!/bin/bash
# gemm4 schedule / memory diagnostics: the same bench under each MFT_G4_DIAG variant (outputs of the
# diagnostic builds are wrong: the error check is skipped with --no_check)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-g4diag}
SH="${2:-8192^3,gpt2 fc fwd}"
mkdir -p $O
cd $R
for d in ${DIAGS:-none nomem nodma spread4 spread2 spread6}; do
  timeout -k 10 120 env MFT_G4_DIAG=$d python3 scripts/bench_gemm4.py --shapes "$SH" --rounds 3 --no_check --only gemm4 > $O/$d.txt 2>&1 || exit 1
done
