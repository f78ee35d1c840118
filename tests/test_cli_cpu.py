"""End-to-end CLI runs on CPU with tiny random-init models + synthetic data (the reference tested
its CLIs by hand with real checkpoints; these pin the behaviour path-free)."""
import json
import os

import pytest
import torch

CPU = ["--device", "cpu", "--dtype", "fp32", "--random_init", "--synthetic_data", "--synthetic_tokens", "20000"]


def test_gpt2_lora_cli_and_resume(tmp_path):
    from mobilefinetuner_amd.cli import gpt2_lora_finetune as cli
    out = str(tmp_path / "lora.safetensors")
    st = str(tmp_path / "state")
    tr = cli.main(["--model", "gpt2-tiny", *CPU, "--steps", "6", "--batch_size", "2", "--seq_len", "32",
                   "--lora_out", out, "--state_dir", st, "--save_every", "3", "--eval_interval", "6",
                   "--eval_batches", "2", "--eval_out", str(tmp_path / "eval.jsonl"), "--log_interval", "1",
                   "--lr", "1e-3", "--lora_targets", "AttnQKV,AttnProj,MlpFcIn,MlpFcOut"])
    assert os.path.exists(out) and os.path.exists(str(tmp_path / "lora_step3.safetensors"))
    recs = [json.loads(x) for x in open(tmp_path / "eval.jsonl")]
    assert recs[0]["step"] == 6 and recs[0]["valid_ppl"] > 1
    assert len(tr.history) == 6
    assert not os.path.exists(st + ".tmp") and not os.path.exists(st + ".old")  # swapped in cleanly
    # a crash between the save's two renames leaves only <state>.old: resume still finds it
    os.rename(st, st + ".old")
    # full-state resume continues at step 6 and runs to 8
    tr2 = cli.main(["--model", "gpt2-tiny", *CPU, "--steps", "8", "--batch_size", "2", "--seq_len", "32",
                    "--resume_from", st, "--lora_targets", "AttnQKV,AttnProj,MlpFcIn,MlpFcOut", "--lr", "1e-3"])
    assert tr2.history[0]["step"] == 7 and len(tr2.history) == 2


def test_gpt2_full_cli(tmp_path):
    from mobilefinetuner_amd.cli import gpt2_full_finetune as cli
    from mobilefinetuner_amd.io import safetensors as st
    out = str(tmp_path / "full.safetensors")
    tr = cli.main(["--model", "gpt2-tiny", *CPU, "--steps", "3", "--batch_size", "2", "--seq_len", "32",
                   "--output_path", out, "--lr", "1e-3"])
    sd = st.load_file(out)
    assert "h.0.attn.c_attn.weight" in sd and sd["wte.weight"].shape == (1000, 128)
    assert tr.total_tokens == 3 * 2 * 32
    state = str(tmp_path / "fstate")
    common = ["--model", "gpt2-tiny", *CPU, "--batch_size", "2", "--seq_len", "32", "--lr", "1e-3", "--state_dir", state]
    cli.main(common + ["--steps", "3"])
    tr2 = cli.main(common + ["--steps", "5"])
    assert [h["step"] for h in tr2.history] == [4, 5] and tr2.total_tokens == 5 * 2 * 32


def test_gemma_cli_and_alignment(tmp_path):
    from mobilefinetuner_amd.cli import train_lora_gemma as cli
    from mobilefinetuner_amd.io.lora_checkpoint import load_lora
    tr = cli.main(["--model", "gemma3-tiny", *CPU, "--max_steps", "4", "--batch", "2", "--seq_len", "32",
                   "--output_dir", str(tmp_path), "--learning_rate", "1e-3", "--targets", "full"])
    t, meta = load_lora(str(tmp_path / "gemma_lora.safetensors"))
    assert meta["targets"] == "attn.q,attn.k,attn.v,attn.proj,mlp.gate,mlp.up,mlp.down"
    assert t["layer.0.attn.q.lora_A"].shape == (8, 128) and t["layer.0.attn.q.lora_B"].shape == (256, 8)
    assert len(tr.history) == 4
    # --state_dir: written at the end, resumed by the next launch (steps 5-6 only)
    sd = str(tmp_path / "gstate")
    common = ["--model", "gemma3-tiny", *CPU, "--batch", "2", "--seq_len", "32", "--output_dir", str(tmp_path / "g2"),
              "--learning_rate", "1e-3", "--targets", "full", "--state_dir", sd]
    cli.main(common + ["--max_steps", "4"])
    tr2 = cli.main(common + ["--max_steps", "6"])
    assert [h["step"] for h in tr2.history] == [5, 6]
    d = str(tmp_path / "align")
    cli.main(["--model", "gemma3-tiny", *CPU, "--batch", "2", "--seq_len", "16", "--align_dump_dir", d,
              "--align_layers", "0,2", "--align_dump_grads", "--align_do_step", "--align_numeric_attn",
              "--align_numeric_count", "2"])
    assert os.path.exists(os.path.join(d, "layer2_mlp_out.npy")) and os.path.isdir(os.path.join(d, "post_step"))


def test_eval_ppl_cli(tmp_path):
    from mobilefinetuner_amd.cli import eval_ppl
    rec = eval_ppl.main(["--model", "gpt2-tiny", *CPU, "--seq_len", "64", "--batch_size", "4",
                         "--out", str(tmp_path / "ppl.jsonl"), "--max_batches", "3"])
    assert rec["task"] == "wt2_ppl" and rec["tokens"] > 0 and rec["ppl"] > 1


def test_eval_mmlu_cli(tmp_path):
    from mobilefinetuner_amd.cli import eval_mmlu
    from tokenizers import Tokenizer, models, pre_tokenizers, trainers
    tok = Tokenizer(models.BPE())
    tok.pre_tokenizer = pre_tokenizers.ByteLevel(add_prefix_space=False)
    tr = trainers.BpeTrainer(vocab_size=300, special_tokens=["<|endoftext|>"],
                             initial_alphabet=pre_tokenizers.ByteLevel.alphabet(), show_progress=False)
    tok.train_from_iterator(["Question: what is A. B. C. D. Answer: "], tr)
    tdir = tmp_path / "tok"
    tdir.mkdir()
    tok.model.save(str(tdir))
    dev = tmp_path / "mmlu" / "dev"
    dev.mkdir(parents=True)
    with open(dev / "astro.csv", "w") as f:
        f.write("subject,question,a,b,c,d,answer\n")
        for i in range(5):
            f.write(f"astro,What is {i}?,x,y,z,w,{'ABCD'[i % 4]}\n")
    res = eval_mmlu.main(["--mmlu_root", str(tmp_path / "mmlu"), "--split", "dev", "--fewshot", "2",
                          "--tokenizer_dir", str(tdir), "--model", "gpt2-tiny", "--device", "cpu", "--dtype", "fp32",
                          "--random_init", "--out", str(tmp_path / "m.jsonl")])
    assert res["total"] == 5 and 0.0 <= res["micro"] <= 1.0


def test_pretokenize_cli_matches_text_mode(tmp_path):
    """cli.pretokenize writes the .bin + meta.json that --pretokenized_path reads, with exactly the
    token stream text mode builds (reference scripts/pretokenize_wikitext2_gemma.py)."""
    import numpy as np
    from tokenizers import Tokenizer, models, pre_tokenizers, trainers
    from mobilefinetuner_amd.cli import pretokenize
    from mobilefinetuner_amd.data.wikitext2 import LMDataset, WT2Config
    from mobilefinetuner_amd.tokenizers import GPT2Tokenizer
    tok = Tokenizer(models.BPE())
    tok.pre_tokenizer = pre_tokenizers.ByteLevel(add_prefix_space=False)
    text = [" = Heading = ", "", " Some text , with numbers 12 and words .", " more words here ."]
    tr = trainers.BpeTrainer(vocab_size=300, special_tokens=["<|endoftext|>"],
                             initial_alphabet=pre_tokenizers.ByteLevel.alphabet(), show_progress=False)
    tok.train_from_iterator(text * 10, tr)
    tdir = tmp_path / "tok"
    tdir.mkdir()
    tok.model.save(str(tdir))
    data = tmp_path / "wt2"
    data.mkdir()
    for split, n in (("train", 30), ("valid", 5), ("test", 3)):
        (data / f"wiki.{split}.raw").write_text("\n".join(text * n) + "\n")
    out = tmp_path / "pt"
    assert pretokenize.main(["--data_dir", str(data), "--tokenizer_dir", str(tdir), "--model_type", "gpt2",
                             "--out_dir", str(out)]) == 0
    meta = json.load(open(out / "meta.json"))
    stream = np.fromfile(out / "wt2_gpt2_tokens.bin", dtype=np.int32)
    assert meta["total_tokens"] == stream.size and set(meta["splits"]) == {"train", "valid", "test"}
    t = GPT2Tokenizer.from_pretrained(str(tdir))
    cfg = WT2Config(data_dir=str(data), seq_len=1, eos_id=t.eos_id, shuffle_train=False, drop_last=False)
    for split in ("train", "valid", "test"):
        ref = np.asarray(LMDataset.from_text(cfg, split, t).tokens())
        o, n = meta["splits"][split]["offset"], meta["splits"][split]["length"]
        assert np.array_equal(stream[o:o + n], ref), split
    # and the training CLI consumes it
    pcfg = WT2Config(pretokenized_path=str(out / "wt2_gpt2_tokens.bin"), seq_len=16, shuffle_train=False)
    ds = LMDataset.from_pretokenized(pcfg, "valid")
    assert ds.num_sequences() == meta["splits"]["valid"]["length"] // 16 or ds.num_sequences() > 0
