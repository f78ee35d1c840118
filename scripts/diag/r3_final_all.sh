#!/bin/bash
set -o pipefail
bash scripts/diag/r3_final_tests.sh || exit 1
bash scripts/diag/r3_final_bench.sh
