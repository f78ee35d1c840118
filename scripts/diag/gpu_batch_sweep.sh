# micro-batch sweep of the two LoRA headline configs (default 512 x 128 / 256 x 256)
set -o pipefail
mkdir -p gpurun_out
for b in 256 512 1024; do
  timeout -k 10 150 python bench.py --steps 20 --warmup 5 --batch $b >> gpurun_out/sweep_gpt2.jsonl 2>>gpurun_out/sweep.err || exit 1
done
for b in 128 256 512; do
  timeout -k 10 200 python bench.py --config gemma3-270m-lora --steps 15 --warmup 4 --batch $b >> gpurun_out/sweep_gemma.jsonl 2>>gpurun_out/sweep.err || exit 1
done
python3 -c "
import json
for f in ['gpurun_out/sweep_gpt2.jsonl','gpurun_out/sweep_gemma.jsonl']:
    for l in open(f):
        d=json.loads(l); print(d['config']['micro_batch_per_gpu'], d['value'], d['ms_per_step'], d['config']['mfu_bf16_dense'])
"
