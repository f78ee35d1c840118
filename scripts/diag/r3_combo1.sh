#!/bin/bash
set -o pipefail
TESTS="${TESTS:-tests}" bash scripts/diag/r3_session_check.sh || exit 1
bash scripts/diag/r3_attn_nw.sh
