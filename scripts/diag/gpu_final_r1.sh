# round-1 closing check: gpu tests, smoke, both headline benches (with MFU fields), headline kernel stats
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/gputests_final.log 2>&1 || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_final.log 2>&1 || exit 1
timeout -k 10 150 python bench.py --steps 30 --warmup 5 > gpurun_out/bench_final3.jsonl 2>gpurun_out/b1_final.err || exit 1
timeout -k 10 150 python bench.py --config gemma3-270m-lora --steps 30 --warmup 5 >> gpurun_out/bench_final3.jsonl 2>gpurun_out/b2_final.err || exit 1
timeout -k 10 200 python bench.py --config gpt2-full --steps 20 --warmup 5 >> gpurun_out/bench_final3.jsonl 2>gpurun_out/b3_final.err || exit 1
cat gpurun_out/bench_final3.jsonl
