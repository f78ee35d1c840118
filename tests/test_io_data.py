"""SafeTensors IO, reference-compatible LoRA checkpoints, LoRA algebra, datasets (CPU)."""
import json
import os
import struct

import pytest
import torch

from mobilefinetuner_amd.io import safetensors as st
from mobilefinetuner_amd.models.gpt2 import GPT2Config, GPT2Model


def test_safetensors_roundtrip_and_hf_compat(tmp_path):
    import safetensors.torch as hst
    ts = {"a": torch.randn(3, 4), "b": torch.arange(10, dtype=torch.int64), "c": torch.randn(5).bfloat16(),
          "d": torch.randn(2, 2).half()}
    p = str(tmp_path / "x.safetensors")
    st.save_file(p, ts, {"k": "v"})
    back = st.load_file(p)
    for k in ts:
        assert back[k].dtype == ts[k].dtype and torch.equal(back[k], ts[k])
    assert st.load_metadata(p) == {"k": "v"}
    hf = hst.load_file(p)  # the official reader accepts our files
    for k in ts:
        assert torch.equal(hf[k], ts[k])
    p2 = str(tmp_path / "y.safetensors")
    hst.save_file({"z": torch.ones(7)}, p2, metadata={"m": "1"})  # and we read theirs
    assert torch.equal(st.load_file(p2)["z"], torch.ones(7)) and st.load_metadata(p2)["m"] == "1"


def _reference_lora_bytes(state, meta):
    """Re-implementation of LoraSaver::save_safetensors' byte layout (graph/lora_saver.cpp:210-280)."""
    keys = sorted(state)
    off, parts = 0, []
    for k in keys:
        t = state[k]
        n = t.numel() * 4
        parts.append(f'"{k}":{{"dtype":"F32","shape":[{",".join(str(s) for s in t.shape)}],'
                     f'"data_offsets":[{off},{off + n}]}}')
        off += n
    h = "{" + ",".join(parts)
    h += ',"__metadata__":{' + ",".join(f'"{k}":"{v}"' for k, v in meta) + "}}"
    hb = h.encode()
    out = struct.pack("<Q", len(hb)) + hb
    for k in keys:
        out += state[k].float().contiguous().numpy().tobytes()
    return out


def _lora_model(split=False, targets=("AttnQKV", "AttnProj")):
    from mobilefinetuner_amd.peft.lora import LoraSpec, inject_gpt2
    cfg = GPT2Config.preset("gpt2-tiny")
    m = GPT2Model(cfg, dtype=torch.float32, device="cpu", seed=1)
    spec = LoraSpec(rank=4, alpha=8, split_qkv=split, targets=list(targets))
    inject_gpt2(m, spec)
    with torch.no_grad():
        for mod in m.modules():
            for sl in getattr(mod, "lora_slices", []):
                sl.B.normal_(0, 0.05)
    return m


@pytest.mark.parametrize("split", [False, True])
def test_lora_checkpoint_matches_reference_bytes(tmp_path, split):
    from mobilefinetuner_amd.io.lora_checkpoint import save_lora
    m = _lora_model(split)
    p = str(tmp_path / "lora.safetensors")
    save_lora(p, m)
    state = {}
    for mod in m.modules():
        for sl in getattr(mod, "lora_slices", []):
            state[sl.name + ".lora_A"] = sl.A.detach().t()
            state[sl.name + ".lora_B"] = sl.B.detach()
    meta = [("rank", "4"), ("alpha", "8"), ("dropout", "0"), ("split_qkv", "true" if split else "false"),
            ("targets", "AttnQKV,AttnProj")]
    assert open(p, "rb").read() == _reference_lora_bytes(state, meta)


def test_lora_roundtrip_and_merge(tmp_path):
    """graph/test_lora_roundtrip.cpp:112-130 and test_lora_correctness.cpp:101-187."""
    from mobilefinetuner_amd.io.lora_checkpoint import attach_lora, load_lora, save_lora
    from mobilefinetuner_amd.peft.lora import merge_all, set_lora_enabled
    m = _lora_model(targets=("AttnQKV", "AttnProj", "MlpFcIn", "MlpFcOut"))
    ids = torch.randint(0, m.cfg.vocab_size, (2, 16))
    with torch.no_grad():
        y0 = m.logits(ids)
    p = str(tmp_path / "a.safetensors")
    save_lora(p, m)
    m2 = GPT2Model(m.cfg, dtype=torch.float32, device="cpu", seed=1)
    tensors, meta = load_lora(p)
    spec = attach_lora(m2, tensors, meta)
    assert spec.rank == 4 and set(spec.targets) == {"AttnQKV", "AttnProj", "MlpFcIn", "MlpFcOut"}
    with torch.no_grad():
        y1 = m2.logits(ids)
    assert (y0 - y1).abs().max() < 1e-5
    w0 = m2.blocks[0].c_attn.weight.detach().clone()
    merge_all(m2)
    set_lora_enabled(m2, False)
    with torch.no_grad():
        y2 = m2.logits(ids)
    assert (y0 - y2).abs().max() < 1e-4
    merge_all(m2, -1.0)
    assert (m2.blocks[0].c_attn.weight - w0).abs().max() < 1e-6


def test_lora_b_zero_is_noop():
    from mobilefinetuner_amd.peft.lora import LoraSpec, inject_gpt2
    cfg = GPT2Config.preset("gpt2-tiny")
    a = GPT2Model(cfg, dtype=torch.float32, device="cpu", seed=2)
    ids = torch.randint(0, cfg.vocab_size, (1, 9))
    with torch.no_grad():
        y0 = a.logits(ids)
        inject_gpt2(a, LoraSpec(rank=8, alpha=16))
        y1 = a.logits(ids)
    assert (y0 - y1).abs().max() < 1e-6


def test_peft_export(tmp_path):
    from mobilefinetuner_amd.io.lora_checkpoint import export_peft
    m = _lora_model()
    export_peft(str(tmp_path / "peft"), m, "gpt2")
    cfg = json.load(open(tmp_path / "peft" / "adapter_config.json"))
    assert cfg["r"] == 4 and set(cfg["target_modules"]) == {"c_attn", "c_proj"}
    t = st.load_file(str(tmp_path / "peft" / "adapter_model.safetensors"))
    a = t["base_model.model.transformer.h.0.attn.c_attn.lora_A.weight"]
    b = t["base_model.model.transformer.h.0.attn.c_attn.lora_B.weight"]
    assert a.shape == (4, 128) and b.shape == (384, 4)


# ------------------------------------------------------------------ datasets
def _write_corpus(d):
    lines = ["= Title =", "", "first line of text .", "second line , with more words .", ""] * 30
    os.makedirs(d, exist_ok=True)
    for n in ("wiki.train.raw", "wiki.valid.raw", "wiki.test.raw"):
        with open(os.path.join(d, n), "w") as f:
            f.write("\n".join(lines) + "\n")
    return lines


def _toy_tokenizer(tmp_path):
    from tokenizers import Tokenizer, decoders, models, pre_tokenizers, trainers
    tok = Tokenizer(models.BPE())
    tok.pre_tokenizer = pre_tokenizers.ByteLevel(add_prefix_space=False)
    tok.decoder = decoders.ByteLevel()
    tr = trainers.BpeTrainer(vocab_size=400, special_tokens=["<|endoftext|>"],
                             initial_alphabet=pre_tokenizers.ByteLevel.alphabet(), show_progress=False)
    tok.train_from_iterator(["first line of text .", "second line , with more words .", "= Title ="], tr)
    d = tmp_path / "tok"
    d.mkdir()
    tok.model.save(str(d))
    from mobilefinetuner_amd.tokenizers import GPT2Tokenizer
    return GPT2Tokenizer.from_pretrained(str(d)), tok


def test_wikitext_chunking_matches_reference_semantics(tmp_path):
    from mobilefinetuner_amd.data.wikitext2 import LMDataset, WT2Config
    lines = _write_corpus(str(tmp_path / "wt2"))
    tok, hf = _toy_tokenizer(tmp_path)
    eos = tok.token_id("<|endoftext|>")
    cfg = WT2Config(data_dir=str(tmp_path / "wt2"), seq_len=16, eos_id=eos, pad_id=0, shuffle_train=False)
    ds = LMDataset.from_text(cfg, "train", tok)
    # expected stream: encode(line) + EOS for every line (blank ones too), trailing EOS ensured
    exp = []
    for ln in lines:
        exp += hf.encode(ln).ids + [eos]
    assert ds.tokens().tolist() == exp
    n_chunks = (len(exp) - 17) // 16 + 1
    assert ds.num_sequences() == n_chunks
    b = ds.next_batch(3)
    ids, tg, mk = b["input_ids"], b["targets"], b["attention_mask"]
    assert ids[0].tolist() == exp[:16] and ids[1].tolist() == exp[16:32]
    assert tg[0, :15].tolist() == exp[1:16] and tg[0, 15].item() == -100  # S-1 predictions per chunk
    assert mk.sum().item() == 48


def test_dataset_tail_shuffle_and_dp_shards(tmp_path):
    from mobilefinetuner_amd.data.wikitext2 import LMDataset, WT2Config
    toks = torch.randint(0, 1 << 30, (1000,), generator=torch.Generator().manual_seed(0), dtype=torch.int64).int()
    cfg = WT2Config(seq_len=64, drop_last=False, shuffle_train=True, seed=7)
    ds = LMDataset(cfg, "valid", toks)
    assert ds.num_sequences() == (1000 - 65) // 64 + 1 + 1  # + padded tail chunk
    tr1 = LMDataset(WT2Config(seq_len=8, seed=7), "train", toks)
    tr2 = LMDataset(WT2Config(seq_len=8, seed=7), "train", toks)
    assert torch.equal(tr1.next_batch(5)["input_ids"], tr2.next_batch(5)["input_ids"])  # deterministic order
    # disjoint equal-sized shards for 3 ranks
    seen = []
    for r in range(3):
        d = LMDataset(WT2Config(seq_len=8, seed=7, rank=r, world=3), "train", toks)
        assert d.num_local() == d.num_sequences() // 3
        rows = []
        while True:
            b = d.next_batch(16, need_loop=False)
            if b is None:
                break
            rows += [tuple(x) for x in b["input_ids"][: b["rows"]].tolist()]
        seen.append(set(rows))
    assert not (seen[0] & seen[1]) and not (seen[1] & seen[2])


def test_dataset_resume_state():
    from mobilefinetuner_amd.data.wikitext2 import LMDataset, WT2Config
    toks = torch.randint(0, 500, (5000,), dtype=torch.int32)
    a = LMDataset(WT2Config(seq_len=16, seed=3), "train", toks)
    for _ in range(40):  # crosses an epoch boundary
        a.next_batch(8)
    stt = a.state()
    nxt = a.next_batch(8)["input_ids"]
    b = LMDataset(WT2Config(seq_len=16, seed=3), "train", toks)
    b.restore(stt)
    assert torch.equal(b.next_batch(8)["input_ids"], nxt)


def test_pretokenized_roundtrip(tmp_path):
    from mobilefinetuner_amd.data.wikitext2 import LMDataset, WT2Config, write_pretokenized
    tr = torch.randint(0, 100, (700,), dtype=torch.int32)
    va = torch.randint(0, 100, (300,), dtype=torch.int32)
    path = write_pretokenized(str(tmp_path / "pt"), {"train": tr, "valid": va}, eos_id=1, pad_id=0, vocab_size=100)
    cfg = WT2Config(pretokenized_path=path, seq_len=32, shuffle_train=False)
    ds = LMDataset.load(cfg, "valid")
    assert torch.equal(ds.tokens(), va)
    assert cfg.eos_id == 1
