"""Native C++ engine (libmft, mobilefinetuner_amd/bin/*) on the GPU.

* engine_selftest: every generic op of the engine's catalog (and its autograd backward) against a
  host fp64 oracle, the caching allocator and the autograd tape semantics (accumulation, hooks).
* Python-path parity: the native ``gpt2_lora_finetune`` CLI and the PyTorch-driven package train
  the SAME random-init GPT-2-124M + LoRA (weights / adapter exchanged through the reference
  safetensors formats) on the SAME pretokenized batches for 10 steps; per-step losses must agree.
* LoRA checkpoint written by the native CLI is byte-identical to the Python writer's file.
"""
import json
import os
import subprocess

import pytest
import torch
from native_logs import loss_list, native_losses

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "mobilefinetuner_amd", "bin")


def _bin(name):
    p = os.path.join(BIN, name)
    if not os.path.exists(p):
        pytest.fail(f"{p} missing: run python -m mobilefinetuner_amd._build")
    return p


def test_engine_selftest():
    r = subprocess.run([_bin("engine_selftest")], capture_output=True, text=True, timeout=180)
    print(r.stdout[-4000:])
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "ALL OK" in r.stdout


def _make_fixture(tmp, S=128, n_tokens=400_000):
    """Random-init GPT-2-124M with perturbed norms / biases and a LoRA adapter whose B is non-zero,
    exported in the HF and reference LoRA formats, plus a pretokenized token stream."""
    from mobilefinetuner_amd.data.wikitext2 import write_pretokenized
    from mobilefinetuner_amd.io import safetensors as st
    from mobilefinetuner_amd.io.lora_checkpoint import save_lora
    from mobilefinetuner_amd.models.gpt2 import GPT2Config, GPT2Model
    from mobilefinetuner_amd.models.hf_io import export_gpt2_state
    from mobilefinetuner_amd.peft.lora import LoraSpec, inject_gpt2

    cfg = GPT2Config.preset("gpt2")
    model = GPT2Model(cfg, device="cuda", seed=1234)
    g = torch.Generator().manual_seed(7)
    with torch.no_grad():
        for b in model.blocks:
            for ln in (b.ln_1, b.ln_2):
                ln.weight.add_((torch.rand(ln.weight.shape, generator=g) - 0.5).cuda() * 0.2)
                ln.bias.add_((torch.rand(ln.bias.shape, generator=g) - 0.5).cuda() * 0.1)
            for lin in (b.c_attn, b.c_proj, b.c_fc, b.mlp_proj):
                lin.bias.copy_(((torch.rand(lin.bias.shape, generator=g) - 0.5) * 0.1).to(lin.bias.dtype).cuda())
    inject_gpt2(model, LoraSpec(rank=8, alpha=16))
    with torch.no_grad():
        for m in model.modules():
            for sl in getattr(m, "lora_slices", []):
                sl.B.copy_(((torch.rand(sl.B.shape, generator=g) - 0.5) * 0.02).cuda())
    os.makedirs(tmp, exist_ok=True)
    st.save_file(os.path.join(tmp, "model.safetensors"), export_gpt2_state(model))
    with open(os.path.join(tmp, "config.json"), "w") as f:
        json.dump({"vocab_size": cfg.vocab_size, "n_positions": cfg.n_positions, "n_embd": cfg.n_embd,
                   "n_layer": cfg.n_layer, "n_head": cfg.n_head}, f)
    lora = os.path.join(tmp, "lora_init.safetensors")
    save_lora(lora, model)
    toks = torch.randint(0, 1000, (n_tokens,), generator=g, dtype=torch.int32)  # learnable: 1000 of 50257 ids
    write_pretokenized(tmp, {"train": toks, "valid": toks[: 40 * (S + 1)]}, eos_id=50256, pad_id=50256,
                       vocab_size=cfg.vocab_size)
    return model, lora


def _python_losses(model, tmp, steps, B, S, lr):
    from mobilefinetuner_amd.data.wikitext2 import LMDataset, WT2Config
    from mobilefinetuner_amd.optim.adamw import FusedAdamW
    from mobilefinetuner_amd.optim.schedules import gpt2_cli_lr
    from mobilefinetuner_amd.peft.lora import lora_parameters
    from mobilefinetuner_amd.train.engine import TrainStep
    from mobilefinetuner_amd.utils.params import FlatParams

    ds = LMDataset.from_pretokenized(WT2Config(pretokenized_path=os.path.join(tmp, "tokens.bin"), seq_len=S,
                                               seed=42), "train")
    flat = FlatParams(lora_parameters(model), "cuda")
    opt = FusedAdamW(flat, lr=lr, weight_decay=0.0, max_grad_norm=1.0)
    step = TrainStep(model, flat, opt, use_graph=True)
    out = []
    for i in range(steps):
        opt.set_lr(gpt2_cli_lr(i, lr, 0, steps))
        b = ds.next_batch(B)
        loss = step([(b["input_ids"].cuda(), b["targets"].cuda())])
        out.append(float(loss.item()))
    return out


def _oracle_trajectory(model, tmp, steps, B, S, lr):
    """The fp32 oracle (tests/oracle host ops): the fixture's weights (bf16 values, exact in fp32) and
    adapter in an fp32 CPU model, trained with torch.optim.AdamW + global-norm clipping on the same
    batches and schedule; returns (per-step losses, adapter state)."""
    from mobilefinetuner_amd.data.wikitext2 import LMDataset, WT2Config
    from mobilefinetuner_amd.io.lora_checkpoint import lora_state
    from mobilefinetuner_amd.models.gpt2 import GPT2Config, GPT2Model
    from mobilefinetuner_amd.optim.schedules import gpt2_cli_lr
    from mobilefinetuner_amd.peft.lora import LoraSpec, inject_gpt2, lora_parameters
    cpu = GPT2Model(GPT2Config.preset("gpt2"), dtype=torch.float32, device="cpu", init=False)
    inject_gpt2(cpu, LoraSpec(rank=8, alpha=16))
    with torch.no_grad():
        src = dict(model.named_parameters())
        for n, p in cpu.named_parameters():
            p.copy_(src[n].detach().float().cpu())
    params = [p for _, p in lora_parameters(cpu)]
    opt = torch.optim.AdamW(params, lr=lr, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0)
    ds = LMDataset.from_pretokenized(WT2Config(pretokenized_path=os.path.join(tmp, "tokens.bin"), seq_len=S,
                                               seed=42), "train")
    out = []
    for i in range(steps):
        for gr in opt.param_groups:
            gr["lr"] = gpt2_cli_lr(i, lr, 0, steps)
        b = ds.next_batch(B)
        opt.zero_grad(set_to_none=True)
        loss = cpu(b["input_ids"], b["targets"])
        loss.backward()
        torch.nn.utils.clip_grad_norm_(params, 1.0)
        opt.step()
        out.append(float(loss.item()))
    return out, lora_state(cpu)[0]


def _update_dev(init, ref, got):
    """rel L2 between two adapters' updates (trained - initial), over every tensor together"""
    num = den = 0.0
    for k in ref:
        d_ref = ref[k].float().cpu() - init[k].float()
        d_got = got[k].float().cpu() - init[k].float()
        num += float((d_ref - d_got).pow(2).sum())
        den += float(d_ref.pow(2).sum())
    assert den > 0, "no update applied"
    return (num / den) ** 0.5


def test_native_cli_matches_python_path(tmp_path):
    """10 LoRA steps of the native CLI against the fp32 oracle's trajectory (losses and the adapter update),
    at a bound set by bf16 rounding itself: the PyTorch-driven bf16 GPU stack trains the same steps, and
    the native engine may deviate from fp32 by at most 1.5x what that other bf16 implementation does
    (+ a 1e-3 loss / 1e-2 update floor) -- a drift in the native path shows, rounding alone does not."""
    S, B, steps, lr = 128, 16, 10, 1e-3
    tmp = str(tmp_path)
    model, lora = _make_fixture(tmp, S)
    from mobilefinetuner_amd.io import safetensors as st
    from mobilefinetuner_amd.io.lora_checkpoint import lora_state
    init = st.load_file(lora)
    ora, ora_state = _oracle_trajectory(model, tmp, steps, B, S, lr)
    py = _python_losses(model, tmp, steps, B, S, lr)
    py_state = lora_state(model)[0]
    metrics = os.path.join(tmp, "native.jsonl")
    out_lora = os.path.join(tmp, "native_lora.safetensors")
    cmd = [_bin("gpt2_lora_finetune"), "--pretrained_dir", tmp, "--resume_from", lora, "--pretokenized_path",
           os.path.join(tmp, "tokens.bin"), "--steps", str(steps), "--batch_size", str(B), "--seq_len", str(S),
           "--lr", str(lr), "--log_interval", "1", "--metrics_out", metrics, "--lora_out", out_lora]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    print(r.stdout[-3000:], r.stderr[-2000:])
    assert r.returncode == 0
    nat = [json.loads(line)["loss"] for line in open(metrics)]
    print("fp32  :", ora)
    print("python:", py)
    print("native:", nat)
    assert len(nat) == steps
    nat_state = st.load_file(out_lora)
    assert sorted(ora_state) == sorted(nat_state) == sorted(py_state)
    d_py, d_nat = _update_dev(init, ora_state, py_state), _update_dev(init, ora_state, nat_state)
    l_py = max(abs(a - b) for a, b in zip(py, ora))
    l_nat = max(abs(a - b) for a, b in zip(nat, ora))
    print(f"vs fp32: loss max|d| python {l_py:.2e} native {l_nat:.2e}; update rel L2 python {d_py:.3e} native {d_nat:.3e}")
    assert l_nat <= 1.5 * l_py + 1e-3, (l_nat, l_py)
    assert d_nat <= 1.5 * d_py + 1e-2, (d_nat, d_py)
    # and the two bf16 paths still see the same per-step losses
    for a, b in zip(py, nat):
        assert abs(a - b) < 2e-3, (py, nat)


def test_native_lora_checkpoint_bytes_match_python(tmp_path):
    """steps=0: the native CLI re-saves the adapter it loaded; the file must equal the Python
    writer's bytes (reference LoraSaver layout: sorted keys, compact header, __metadata__ last)."""
    tmp = str(tmp_path)
    _, lora = _make_fixture(tmp, 64, 20_000)
    out = os.path.join(tmp, "resaved.safetensors")
    r = subprocess.run([_bin("gpt2_lora_finetune"), "--pretrained_dir", tmp, "--resume_from", lora,
                        "--pretokenized_path", os.path.join(tmp, "tokens.bin"), "--steps", "0", "--seq_len", "64",
                        "--lora_out", out], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert open(out, "rb").read() == open(lora, "rb").read()


def test_native_eager_and_graph_agree():
    # --deterministic: fixed-order reductions instead of fp32 atomics, so eager and graph replay must
    # agree to the last printed digit
    common = ["--random_init", "--model", "gpt2-tiny", "--synthetic_data", "--synthetic_tokens", "100000", "--steps",
              "5", "--batch_size", "4", "--seq_len", "64", "--lr", "1e-3", "--log_interval", "1", "--deterministic"]
    outs = []
    for extra in ([], ["--no_graph"]):
        r = subprocess.run([_bin("gpt2_lora_finetune"), *common, *extra], capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
        outs.append(loss_list(r.stdout))
    assert outs[0] == outs[1] and len(outs[0]) == 5


def test_native_full_finetune_runs(tmp_path):
    from mobilefinetuner_amd.io import safetensors as st
    outs = {}
    for steps in (0, 6):
        out = str(tmp_path / f"full{steps}.safetensors")
        r = subprocess.run([_bin("gpt2_full_finetune"), "--random_init", "--model", "gpt2-tiny", "--synthetic_data",
                            "--synthetic_tokens", "100000", "--steps", str(steps), "--batch_size", "4", "--seq_len",
                            "64", "--lr", "1e-3", "--log_interval", "1", "--output_path", out], capture_output=True,
                           text=True, timeout=120)
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
        losses = loss_list(r.stdout, True)
        assert len(losses) == steps and all(l == l and abs(l) < 20 for l in losses)
        outs[steps] = st.load_file(out)
    sd0, sd6 = outs[0], outs[6]
    assert "h.0.attn.c_attn.weight" in sd6 and sd6["wte.weight"].shape == (1000, 128)
    assert sd6["h.0.attn.c_attn.weight"].shape == (128, 384)  # HF Conv1D [in, out]
    # every tensor kind was trained (weights, biases, norms, tied embedding)
    for k in ("wte.weight", "h.1.mlp.c_proj.weight", "h.0.ln_1.weight", "h.0.attn.c_attn.bias", "ln_f.bias"):
        assert not torch.equal(sd0[k], sd6[k]), k


def test_native_cli_with_rccl_communicator():
    """The native data-parallel path (engine/comm.h: RCCL communicator, rank-0 broadcast of the
    trainable weights, gradient all-reduce between the replayed forward/backward graph and the
    optimizer, reduced eval sums) on a 1-rank group (MFT_DP_FORCE_COMM=1): identical losses to the
    single-process run (--deterministic; a 1-rank average is exact)."""
    common = ["--random_init", "--model", "gpt2-tiny", "--synthetic_data", "--synthetic_tokens", "100000", "--steps",
              "6", "--batch_size", "4", "--seq_len", "64", "--lr", "1e-3", "--log_interval", "1", "--deterministic",
              "--eval_interval", "3", "--eval_batches", "4"]
    outs = []
    for force in ("0", "1"):
        env = dict(os.environ, MFT_DP_FORCE_COMM=force, MASTER_ADDR="127.0.0.1", MASTER_PORT="29611")
        env.pop("WORLD_SIZE", None)
        r = subprocess.run([_bin("gpt2_lora_finetune"), *common], capture_output=True, text=True, timeout=180, env=env)
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
        if force == "1":
            assert "data parallel: rank 0 of 1" in r.stdout
        steps = loss_list(r.stdout)
        evals = [ln for ln in r.stdout.splitlines() if ln.startswith("[Eval]")]
        outs.append((steps, evals))
    assert outs[0] == outs[1] and len(outs[0][0]) == 6 and len(outs[0][1]) == 2, outs


def test_native_eval_ppl_matches_python_cli(tmp_path):
    """Native eval_ppl (fused LM head, merged LoRA) == the Python eval_ppl CLI on the same weights,
    adapter and pretokenized validation split."""
    tmp = str(tmp_path)
    _, lora = _make_fixture(tmp, 128, 60_000)
    common = ["--pretrained_dir", tmp, "--lora_path", lora, "--pretokenized_path", os.path.join(tmp, "tokens.bin"),
              "--split", "valid", "--seq_len", "128", "--batch_size", "4"]
    nat_out, py_out = os.path.join(tmp, "nat.json"), os.path.join(tmp, "py.json")
    r = subprocess.run([_bin("eval_ppl"), *common, "--out", nat_out], capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    env = dict(os.environ, PYTHONPATH=ROOT)
    r = subprocess.run(["python", "-m", "mobilefinetuner_amd.cli.eval_ppl", *common, "--out", py_out],
                       capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    nat, py = json.load(open(nat_out)), json.loads(open(py_out).read().splitlines()[-1])
    print(nat, py)
    assert nat["tokens"] == py.get("tokens", py.get("n_tokens", nat["tokens"]))
    assert abs(nat["ppl"] - py["ppl"]) < 2e-3 * py["ppl"], (nat, py)


def test_native_weight_streaming_matches_resident(tmp_path):
    """--shard_enable in the native CLI: GPT-2's frozen block weights in pinned host memory, streamed
    through 2 device slots (40 MB budget, 14 MB per block) with prefetch and backward re-loads, in the
    hipGraph-captured step and eagerly -- the same per-step losses as the resident run.  With
    --shard_dir the blocks live in files (fp16 by default, --shard_fp16_disk 0: bf16) read by host
    nodes of the copy stream: same losses (bf16 -> fp16 -> bf16 is exact for these weights)."""
    common = ["--random_init", "--model", "gpt2", "--synthetic_data", "--synthetic_tokens", "200000", "--steps", "6",
              "--batch_size", "4", "--seq_len", "64", "--lr", "1e-3", "--log_interval", "1", "--deterministic"]

    def losses(extra):
        r = subprocess.run([_bin("gpt2_lora_finetune"), *common, *extra], capture_output=True, text=True, timeout=180)
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
        return loss_list(r.stdout, True), r.stdout

    ref, _ = losses([])
    d16, d = str(tmp_path / "fp16"), str(tmp_path / "bf16")
    for extra in ([], ["--no_graph"], ["--shard_dir", d16], ["--shard_dir", d, "--shard_fp16_disk", "0", "--no_graph"]):
        got, out = losses(["--shard_enable", "--shard_budget_mb", "40", *extra])
        assert "weight streaming ON: 2 device slots" in out, out[-2000:]
        if extra and extra[0] == "--shard_dir":
            assert "on disk" in out, out[-2000:]
            files = sorted(os.listdir(extra[1]))
            assert len(files) == 12 and all(f.startswith("block_") for f in files), files
            assert os.path.getsize(os.path.join(extra[1], "block_0.bin")) >= 7_000_000 * 2
        assert len(got) == 6 and got == pytest.approx(ref, abs=2e-3), (extra, got, ref)


@pytest.mark.parametrize("prog,model,steps_flag,extra", [
    ("gpt2_lora_finetune", "gpt2-tiny", "--steps", ["--batch_size", "4", "--warmup_steps", "100", "--lora_dropout", "0.1"]),
    ("train_lora_gemma", "gemma3-tiny", "--max_steps", ["--batch", "4", "--lr_schedule", "constant",
                                                        "--lora_dropout", "0.1"]),
    # full fine-tune with the AdamW moments on disk (--offload disk): saved from / restored into the file mappings
    ("gpt2_full_finetune", "gpt2-tiny", "--steps", ["--batch_size", "4", "--warmup_steps", "100", "--offload", "disk",
                                                    "--offload_moments", "fp32", "--offload_dir", "{tmp}/offload"]),
])
def test_native_full_state_resume(tmp_path, prog, model, steps_flag, extra):
    """--state_dir: 4 steps, then a fresh process resumes from the saved state (fp32 master, AdamW
    moments + step, data cursor / shuffle RNG, EMA, LoRA-dropout counter) and runs steps 5-8; its
    losses equal the uninterrupted 8-step run's (deterministic mode; the schedule is chosen so the
    learning rate does not depend on the run's total step count)."""
    extra = [x.replace("{tmp}", str(tmp_path)) for x in extra]
    common = [_bin(prog), "--random_init", "--model", model, "--synthetic_data", "--synthetic_tokens", "100000",
              "--seq_len", "64", "--lr", "1e-3", "--log_interval", "1", "--deterministic", *extra]

    def losses(steps, state=None):
        cmd = common + [steps_flag, str(steps)] + (["--state_dir", state] if state else [])
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=180)
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
        return r.stdout, native_losses(r.stdout)

    _, ref = losses(8)
    state = str(tmp_path / "state")
    _, first = losses(4, state)
    assert os.path.exists(os.path.join(state, "optimizer.safetensors"))
    st = json.load(open(os.path.join(state, "trainer_state.rank0.json")))
    assert st["global_step"] == 4 and st["opt_step"] == 4
    out, second = losses(8, state)
    assert "resumed full training state" in out
    assert sorted(first) == [1, 2, 3, 4] and sorted(second) == [5, 6, 7, 8]
    assert [first[i] for i in range(1, 5)] == [ref[i] for i in range(1, 5)]
    assert [second[i] for i in range(5, 9)] == [ref[i] for i in range(5, 9)], (ref, first, second)


def test_native_fault_then_resume(tmp_path):
    """SURVEY §5.3 failure path: --inject_fault 6:0 kills the run before step 6 (non-zero exit, the
    state of step 4 from --save_every on disk); relaunching the same command without the fault resumes
    at step 5 and finishes with the uninterrupted run's losses."""
    state = str(tmp_path / "state")
    common = [_bin("gpt2_lora_finetune"), "--random_init", "--model", "gpt2-tiny", "--synthetic_data",
              "--synthetic_tokens", "100000", "--batch_size", "4", "--seq_len", "64", "--lr", "1e-3",
              "--warmup_steps", "100", "--log_interval", "1", "--deterministic", "--steps", "8"]

    def run(extra):
        return subprocess.run(common + extra, capture_output=True, text=True, timeout=180)

    def losses(out):
        return native_losses(out)

    r = run([])
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    ref = losses(r.stdout)
    r = run(["--save_every", "4", "--state_dir", state, "--inject_fault", "6:0"])
    assert r.returncode != 0 and "injected fault at step 6" in r.stderr, r.stdout[-1000:] + r.stderr[-1000:]
    assert sorted(losses(r.stdout)) == [1, 2, 3, 4, 5]
    assert json.load(open(os.path.join(state, "trainer_state.rank0.json")))["global_step"] == 4
    r = run(["--save_every", "4", "--state_dir", state])
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    got = losses(r.stdout)
    assert sorted(got) == [5, 6, 7, 8] and all(got[i] == ref[i] for i in got), (ref, got)


def test_native_common_flag_block(tmp_path):
    """The native CLIs' common flag block:
    * --attn_impl naive (materialized masked softmax) trains like the flash kernels (bf16 noise);
    * --dtype fp32 (reference-precision composite path, eager) trains and tracks the bf16 run;
    * --profile_steps a:b prints one device time per step of the window and nothing else;
    * --compat_grad_overwrite keeps only the last micro-batch's gradient (reference Q1): with two
      micro-batches the first step's update differs from the accumulating run's."""
    common = ["--random_init", "--model", "gpt2-tiny", "--synthetic_data", "--synthetic_tokens", "100000", "--steps",
              "6", "--batch_size", "4", "--seq_len", "64", "--lr", "1e-3", "--log_interval", "1", "--deterministic"]

    def run(extra, prog="gpt2_lora_finetune"):
        r = subprocess.run([_bin(prog), *common, *extra], capture_output=True, text=True, timeout=180)
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
        return loss_list(r.stdout, True), r.stdout

    ref, _ = run([])
    naive, out = run(["--attn_impl", "naive"])
    assert "step runs eagerly" in out
    assert naive == pytest.approx(ref, abs=2e-2), (naive, ref)
    f32, out = run(["--dtype", "fp32"])
    assert "--dtype fp32" in out and all(x == x for x in f32)
    assert f32 == pytest.approx(ref, abs=3e-2), (f32, ref)
    _, out = run(["--profile_steps", "2:4"])
    prof = [ln for ln in out.splitlines() if ln.startswith("[profile] step ")]
    assert [int(ln.split()[2].rstrip(":")) for ln in prof] == [2, 3, 4], prof
    acc, _ = run(["--grad_accum_steps", "2"])
    ow, _ = run(["--grad_accum_steps", "2", "--compat_grad_overwrite"])
    assert acc[0] == pytest.approx(ow[0], abs=1e-6)  # the same first forward
    assert ow[1:] != acc[1:]  # different updates from then on
    # full fine-tuning in fp32 (every weight an fp32 leaf, tied embedding through both uses)
    full, _ = run(["--dtype", "fp32"], prog="gpt2_full_finetune")
    full_bf16, _ = run([], prog="gpt2_full_finetune")
    assert len(full) == 6 and full == pytest.approx(full_bf16, abs=3e-2), (full, full_bf16)
