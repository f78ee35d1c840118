"""Native eval_mmlu (mobilefinetuner_amd/bin/eval_mmlu) vs the Python MMLU evaluator on the GPU:
same CSV reading (quoted fields with commas / quotes, headered and headerless files), same prompts
(k-shot, the item never its own example), same letter log-probs per question (the native
--scores_out against eval.mmlu.score_prompts on identical random-init GPT-2 weights), same accuracy
wherever the prediction is not a near-tie."""
import json
import os
import subprocess

import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "mobilefinetuner_amd", "bin")


def _fixture(tmp):
    from tokenizers import Tokenizer, models, pre_tokenizers, trainers
    from mobilefinetuner_amd.io import safetensors as st
    from mobilefinetuner_amd.models.gpt2 import GPT2Config, GPT2Model
    from mobilefinetuner_amd.models.hf_io import export_gpt2_state
    tok = Tokenizer(models.BPE())
    tok.pre_tokenizer = pre_tokenizers.ByteLevel(add_prefix_space=False)
    tr = trainers.BpeTrainer(vocab_size=300, special_tokens=["<|endoftext|>"],
                             initial_alphabet=pre_tokenizers.ByteLevel.alphabet(), show_progress=False)
    tok.train_from_iterator(["Question: what is the value of x, y and z? A. B. C. D. Answer: "] * 20, tr)
    tok.model.save(tmp)
    cfg = GPT2Config.preset("gpt2-tiny")
    model = GPT2Model(cfg, device="cuda", seed=11)
    st.save_file(os.path.join(tmp, "model.safetensors"), export_gpt2_state(model))
    with open(os.path.join(tmp, "config.json"), "w") as f:
        json.dump({"vocab_size": cfg.vocab_size, "n_positions": cfg.n_positions, "n_embd": cfg.n_embd,
                   "n_layer": cfg.n_layer, "n_head": cfg.n_head}, f)
    dev = os.path.join(tmp, "mmlu", "dev")
    os.makedirs(dev)
    with open(os.path.join(dev, "astronomy_dev.csv"), "w") as f:  # headered, quoted fields
        f.write("subject,question,a,b,c,d,answer\n")
        for i in range(11):
            f.write(f'astronomy,"What is {i}, really?",x{i},"y ""{i}""",z,w,{"ABCD"[i % 4]}\n')
    with open(os.path.join(dev, "algebra_dev.csv"), "w") as f:  # headerless Hendrycks layout
        for i in range(7):
            f.write(f"Solve {i} + x = {2 * i}.,{i},{2 * i},{3 * i},x,{'DCBA'[i % 4]}\n")
    return model


def test_native_eval_mmlu_matches_python(tmp_path):
    from mobilefinetuner_amd.eval.mmlu import build_prompt, read_split, score_prompts
    from mobilefinetuner_amd.tokenizers import GPT2Tokenizer
    tmp = str(tmp_path)
    model = _fixture(tmp)
    exe = os.path.join(BIN, "eval_mmlu")
    assert os.path.exists(exe), "run python -m mobilefinetuner_amd._build"
    scores = os.path.join(tmp, "scores.txt")
    r = subprocess.run([exe, "--mmlu_root", os.path.join(tmp, "mmlu"), "--split", "dev", "--fewshot", "2",
                        "--pretrained_dir", tmp, "--batch_size", "4", "--scores_out", scores,
                        "--out", os.path.join(tmp, "nat.jsonl")], capture_output=True, text=True, timeout=180)
    print(r.stdout[-2000:], r.stderr[-2000:])
    assert r.returncode == 0
    nat = torch.tensor([[float(x) for x in line.split()] for line in open(scores)])
    res = json.loads(r.stdout.strip().splitlines()[-1])
    # Python side: same prompts in the same (subject-sorted) order
    tok = GPT2Tokenizer.from_pretrained(tmp)
    data = read_split(os.path.join(tmp, "mmlu"), "dev")
    letters = [tok.encode(L)[0] for L in "ABCD"]
    model.eval()
    py, answers = [], []
    for subj in sorted(data):
        items = data[subj]
        prompts = [build_prompt(x, [items[j] for j in range(min(2, len(items))) if j != i]) for i, x in enumerate(items)]
        py.append(score_prompts(model, tok, prompts, letters, torch.device("cuda"), 4, model.cfg.n_positions))
        answers += [x.answer for x in items]
    py = torch.cat(py)
    assert nat.shape == py.shape == (18, 4) and res["total"] == 18
    assert (nat - py).abs().max().item() < 3e-2, (nat - py).abs().max().item()
    top2 = py.topk(2, dim=1).values
    clear = (top2[:, 0] - top2[:, 1]) > 0.05
    assert torch.equal(nat.argmax(1)[clear], py.argmax(1)[clear])
    micro_py = sum("ABCD"[p] == a for p, a in zip(py.argmax(1).tolist(), answers)) / len(answers)
    if bool(clear.all()):
        assert abs(res["micro"] - micro_py) < 1e-9
