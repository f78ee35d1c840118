#!/bin/bash
set -o pipefail
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 200 python3 scripts/diag/rs_tail.py 2>&1 | grep -E "^n=" | tail -50
