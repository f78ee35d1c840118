#!/bin/bash
# native-engine bench.py runs (the driver's default path) + the ZeRO-3 gradient-zeroing test
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r3_nb_gpt2.json 2> gpurun_out/r3_nb_gpt2.err || { tail -20 gpurun_out/r3_nb_gpt2.err; exit 1; }
cat gpurun_out/r3_nb_gpt2.json
timeout -k 10 200 python3 bench.py --config gemma3-270m-lora --steps 15 --warmup 4 > gpurun_out/r3_nb_gemma.json 2> gpurun_out/r3_nb_gemma.err || { tail -20 gpurun_out/r3_nb_gemma.err; exit 1; }
cat gpurun_out/r3_nb_gemma.json
timeout -k 10 200 python3 bench.py --config gpt2-full --steps 15 --warmup 4 > gpurun_out/r3_nb_full.json 2> gpurun_out/r3_nb_full.err || { tail -20 gpurun_out/r3_nb_full.err; exit 1; }
cat gpurun_out/r3_nb_full.json
timeout -k 10 200 python3 bench.py --config gpt2-full --engine torch --steps 15 --warmup 4 > gpurun_out/r3_tb_full.json 2> gpurun_out/r3_tb_full.err || { tail -20 gpurun_out/r3_tb_full.err; exit 1; }
cat gpurun_out/r3_tb_full.json
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_models_gpu.py -k zero3 > gpurun_out/r3_z3_test.log 2>&1 || { tail -30 gpurun_out/r3_z3_test.log; exit 1; }
tail -3 gpurun_out/r3_z3_test.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3_smoke.log 2>&1 || { tail -30 gpurun_out/r3_smoke.log; exit 1; }
tail -3 gpurun_out/r3_smoke.log
