#!/bin/bash
# GEMM routing maps of every bench config (MFT_GEMM_MAP=1: one line per shape and backend) and the
# headline's kernel table
set -o pipefail
O=gpurun_out/${1:-r5map}
mkdir -p $O
export TMPDIR=/tmp
for c in gpt2-lora gemma3-270m-lora gemma3-1b-lora gpt2-full gpt2-xl-zero3; do
  MFT_GEMM_MAP=1 timeout -k 10 300 python3 bench.py --config $c --steps 3 --warmup 1 > $O/map_$c.txt 2>&1 || { tail -5 $O/map_$c.txt; exit 1; }
  echo "== $c"; grep "gemm-map" $O/map_$c.txt | sort | uniq
done
B4="--random_init --synthetic_data --synthetic_tokens 2000000 --seq_len 128 --batch_size 4 --steps 12 --log_interval 0 --bench_steps 4 --bench_warmup 4 --no_graph"
MFT_GEMM_MAP=1 timeout -k 10 300 mobilefinetuner_amd/bin/gpt2_lora_finetune $B4 > $O/map_b4.txt 2>&1 || { tail -5 $O/map_b4.txt; exit 1; }
echo "== gpt2-lora batch 4 x 128 (short tokens, eager)"; grep "gemm-map" $O/map_b4.txt | sort | uniq
A="--random_init --synthetic_data --synthetic_tokens 2000000 --seq_len 128 --batch_size 1024 --steps 14 --log_interval 0 --bench_steps 6 --bench_warmup 4"
rm -rf $O/p_g2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p_g2 -o run -- mobilefinetuner_amd/bin/gpt2_lora_finetune $A > $O/g2_prof.log 2>&1 || { tail -5 $O/g2_prof.log; exit 1; }
DB=$(find $O/p_g2 -name "*.db" | head -1)
python3 scripts/prof_db.py $DB stats 10 40 > $O/gpt2_lora_kernel_stats.txt && head -24 $O/gpt2_lora_kernel_stats.txt | cut -c1-150
rm -rf $O/p_g2
