#!/bin/bash
# round-3 re-entry check of the restored tree: every GPU test + smoke, the two LoRA benches and a
# kernel profile of the native Gemma-3 step (256 x 256)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 900 python3 -u -m pytest ${TESTS:-tests} -m gpu -q --timeout 400 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r3s_gpu_tests.log 2>&1; rc=$?; echo "gpu tests rc=$rc"
grep -E "passed|failed" gpurun_out/r3s_gpu_tests.log | tail -2; grep -E "^FAILED" gpurun_out/r3s_gpu_tests.log | head
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3s_smoke.log 2>&1 || { tail gpurun_out/r3s_smoke.log; exit 1; }
tail -1 gpurun_out/r3s_smoke.log
rm -f gpurun_out/r3s_bench.jsonl
for cfg in gpt2-lora gemma3-270m-lora gpt2-full; do
  timeout -k 10 300 python3 bench.py --config $cfg --steps 20 --warmup 5 >> gpurun_out/r3s_bench.jsonl 2> gpurun_out/r3s_$cfg.err || { tail -20 gpurun_out/r3s_$cfg.err; exit 1; }
  echo "$cfg: $(tail -1 gpurun_out/r3s_bench.jsonl | cut -c1-170)"
done
rm -rf gpurun_out/p_gemma
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/p_gemma -o run -- mobilefinetuner_amd/bin/train_lora_gemma \
  --model gemma3-270m --random_init --synthetic_data --synthetic_tokens 2000000 --batch 256 --seq_len 256 --lora_dropout 0 \
  --targets full --max_steps 12 --log_interval 12 > gpurun_out/r3s_gemma_prof.log 2>&1 || { tail gpurun_out/r3s_gemma_prof.log; exit 1; }
DB=$(find gpurun_out/p_gemma -name "*.db" | head -1)
python3 scripts/prof_db.py $DB stats 12 40 > gpurun_out/r3s_gemma_stats.txt
rm -rf gpurun_out/p_gemma
head -24 gpurun_out/r3s_gemma_stats.txt
