#!/bin/bash
set -o pipefail
bash scripts/diag/r3_gemma_prof.sh
bash scripts/diag/r3_attn_nw.sh
