"""Multi-process data parallelism on CPU (gloo, world_size 2): DP gradients equal the single-process
large-batch gradients, ZeRO-1/2 training equals DDP training, and the CLI runs under torchrun-style
env.  (The reference has no distributed code; SURVEY §7.5 asks for these equivalence tests.)"""
import os
import socket
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    sys.path.insert(0, ROOT)
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)


def _model():
    from mobilefinetuner_amd.models.gpt2 import GPT2Config, GPT2Model
    from mobilefinetuner_amd.peft.lora import LoraSpec, inject_gpt2
    m = GPT2Model(GPT2Config.preset("gpt2-tiny"), dtype=torch.float32, device="cpu", seed=5)
    inject_gpt2(m, LoraSpec(rank=4, alpha=8, targets=["AttnQKV", "AttnProj", "MlpFcIn"]))
    with torch.no_grad():
        for mod in m.modules():
            for sl in getattr(mod, "lora_slices", []):
                sl.B.normal_(0, 0.02, generator=torch.Generator().manual_seed(7))
    return m


def _worker_ddp(rank, world, port, q):
    _init(rank, world, port)
    from mobilefinetuner_amd.parallel.ddp import DataParallel
    from mobilefinetuner_amd.peft.lora import lora_parameters
    from mobilefinetuner_amd.utils.params import FlatParams
    m = _model()
    flat = FlatParams(lora_parameters(m), "cpu", shadow=False)
    dp = DataParallel(flat, bucket_mb=0.01)  # tiny buckets -> several async all-reduces
    ids = torch.randint(0, 1000, (4, 17), generator=torch.Generator().manual_seed(3))
    mine = ids[rank * 2:(rank + 1) * 2]
    dp.begin_step()
    flat.grad.zero_()
    loss = m(mine[:, :-1], mine[:, 1:])
    loss.backward()
    dp.finish()
    q.put((rank, flat.grad.clone().numpy(), len(dp.buckets)))
    dist.destroy_process_group()


def test_ddp_grads_equal_single_process_large_batch():
    from mobilefinetuner_amd.peft.lora import lora_parameters
    from mobilefinetuner_amd.utils.params import FlatParams
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker_ddp, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict((r, (torch.as_tensor(g), nb)) for r, g, nb in [q.get(timeout=300) for _ in ps])
    for p in ps:
        p.join(60)
    sys.path.insert(0, ROOT)
    m = _model()
    flat = FlatParams(lora_parameters(m), "cpu", shadow=False)
    ids = torch.randint(0, 1000, (4, 17), generator=torch.Generator().manual_seed(3))
    # mean over ranks of per-rank mean losses == mean loss over the 4 sequences (equal token counts)
    loss = m(ids[:, :-1], ids[:, 1:])
    loss.backward()
    assert res[0][1] > 1, "expected several buckets"
    assert torch.allclose(res[0][0], res[1][0])
    assert torch.allclose(res[0][0], flat.grad, atol=1e-6, rtol=1e-4), (res[0][0] - flat.grad).abs().max()


def _worker_train(rank, world, port, stage, q, accum=1, ckpt=False):
    _init(rank, world, port)
    from mobilefinetuner_amd.data.wikitext2 import LMDataset, WT2Config
    from mobilefinetuner_amd.models.gpt2 import GPT2Config, GPT2Model
    from mobilefinetuner_amd.parallel.ddp import DataParallel
    from mobilefinetuner_amd.train.trainer import TrainConfig, Trainer
    from mobilefinetuner_amd.utils.params import FlatParams
    m = GPT2Model(GPT2Config.preset("gpt2-tiny"), dtype=torch.float32, device="cpu", seed=11)
    m.set_full_finetune()
    m.activation_checkpointing = ckpt
    if stage == 3:
        from mobilefinetuner_amd.parallel.zero3 import attach_zero3
        flat = attach_zero3(m, "cpu").flat
    else:
        flat = FlatParams(m.named_parameters(), "cpu", shadow=False, pad_multiple=world)
    toks = torch.randint(0, 1000, (8000,), generator=torch.Generator().manual_seed(0), dtype=torch.int64).int()
    ds = LMDataset(WT2Config(seq_len=32, seed=1, rank=rank, world=world), "train", toks)
    dp = DataParallel(flat, bucket_mb=0.05) if stage == 0 else None
    tc = TrainConfig(steps=4, batch_size=2, grad_accum=accum, lr=1e-3, weight_decay=0.01, clip_grad_norm=0.5,
                     log_interval=1, use_graph=False, ema_beta=0.0)
    tr = Trainer(m, flat, ds, None, tc, torch.device("cpu"), dp=dp, zero_stage=stage)
    tr.train()
    if stage == 3:
        # between steps no unit is gathered or holds a live gradient buffer, and the blocks share
        # two fixed slots (no allocation inside a step -> graph-capturable)
        z3 = m.zero3
        assert not any(u.gathered or u.g_live for u in z3.units)
        blocks = z3.units[1:]
        assert len({u.full.data_ptr() for u in blocks}) == min(2, len(blocks))
        params = m.zero3.full_state()
    else:
        if stage:
            tr.opt.gather_master()
        params = {n: p.detach().clone() for n, p in m.named_parameters()}
    # numpy arrays pickle by value (shared-memory tensors would die with this process)
    q.put((rank, {n: t.float().numpy().copy() for n, t in params.items()}, [h["loss"] for h in tr.history]))
    dist.destroy_process_group()


def _run_train(stage, accum=1, ckpt=False):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker_train, args=(r, 2, port, stage, q, accum, ckpt)) for r in range(2)]
    for p in ps:
        p.start()
    out = dict((r, ({n: torch.from_numpy(a) for n, a in w.items()}, l)) for r, w, l in [q.get(timeout=600) for _ in ps])
    for p in ps:
        p.join(60)
    return out


@pytest.mark.parametrize("stage,accum,ckpt", [(1, 1, False), (2, 1, False), (3, 1, False), (3, 2, True)])
def test_zero_matches_ddp(stage, accum, ckpt):
    """ZeRO-1/2/3 training (4 steps, clipping + weight decay; ZeRO-3 also with grad accumulation and
    activation checkpointing) == DDP training, on every rank."""
    ddp = _run_train(0, accum)
    zero = _run_train(stage, accum, ckpt)
    assert ddp[0][1] == pytest.approx(zero[0][1], rel=1e-4)
    assert set(zero[0][0]) == set(ddp[0][0])
    for n, w in ddp[0][0].items():
        assert torch.allclose(w, ddp[1][0][n])
        assert torch.allclose(w, zero[0][0][n], atol=1e-5), (n, (w - zero[0][0][n]).abs().max())
        assert torch.allclose(zero[0][0][n], zero[1][0][n])


def test_mft_launch_propagates_rank_failure(tmp_path):
    """a failing rank stops the job (peers blocked in a collective are terminated)."""
    import time
    from mobilefinetuner_amd.launch import launch
    script = tmp_path / "job.py"
    script.write_text(
        "import os, sys, time\n"
        "import torch.distributed as dist\n"
        "dist.init_process_group('gloo')\n"
        "if int(os.environ['RANK']) == 1:\n"
        "    sys.exit(3)\n"
        "dist.barrier()  # rank 0 would wait here forever\n"
        "time.sleep(600)\n")
    t0 = time.time()
    code = launch([str(script)], 2, grace=2.0)
    assert code == 3 and time.time() - t0 < 60
    ok = tmp_path / "ok.py"
    ok.write_text("import os\nassert os.environ['WORLD_SIZE'] == '2' and os.environ['MASTER_ADDR'] == '127.0.0.1'\n")
    assert launch([str(ok)], 2) == 0


def test_cli_inject_fault_under_launcher(tmp_path):
    """--inject_fault step:rank raises on that rank; mft_launch reports the failure and stops rank 0."""
    from mobilefinetuner_amd.launch import launch
    code = launch(["-m", "mobilefinetuner_amd.cli.gpt2_lora_finetune", "--model", "gpt2-tiny", "--device", "cpu",
                   "--dtype", "fp32", "--random_init", "--synthetic_data", "--synthetic_tokens", "20000",
                   "--steps", "6", "--batch_size", "2", "--seq_len", "32", "--lora_out",
                   str(tmp_path / "l.safetensors"), "--inject_fault", "3:1", "--dist_timeout_s", "60"],
                  2, grace=2.0, extra_env={"PYTHONPATH": ROOT, "OMP_NUM_THREADS": "1"})
    assert code != 0


def _worker_zero_shadow(rank, world, port, q):
    _init(rank, world, port)
    from mobilefinetuner_amd.models.gpt2 import GPT2Config, GPT2Model
    from mobilefinetuner_amd.parallel.zero import ZeroOptimizer
    from mobilefinetuner_amd.utils.params import FlatParams
    m = GPT2Model(GPT2Config.preset("gpt2-tiny"), dtype=torch.float32, device="cpu", seed=5)
    m.set_full_finetune()
    # a bf16 shadow as on the GPU: norm weights (no shadow) must still be synchronised across ranks
    flat = FlatParams(m.named_parameters(), "cpu", shadow=True, pad_multiple=world)
    opt = ZeroOptimizer(flat, 2, lr=1e-2, weight_decay=0.0, max_grad_norm=None)
    for _ in range(2):
        flat.grad.normal_(0, 1.0, generator=torch.Generator().manual_seed(rank + 1))
        opt.reduce_gradients()
        opt.step()
    ln = torch.cat([m.blocks[0].ln_1.weight.detach().flatten(), m.ln_f.bias.detach().flatten()])
    q.put((rank, ln.clone().numpy()))
    dist.destroy_process_group()


def test_zero_syncs_fp32_compute_params():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker_zero_shadow, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    out = dict((r, torch.as_tensor(v)) for r, v in [q.get(timeout=600) for _ in ps])
    for p in ps:
        p.join(60)
    assert not torch.equal(out[0], torch.ones_like(out[0]))  # updated
    assert torch.equal(out[0], out[1])


def test_ddp_hook_defers_inside_graph_capture(monkeypatch):
    """A bucket's grad-ready hook must not enqueue a collective while a hipGraph is being captured
    (TrainStep use_graph): the bucket stays pending and finish() reduces it after the replay."""
    sys.path.insert(0, ROOT)
    from mobilefinetuner_amd.parallel.ddp import DataParallel
    from mobilefinetuner_amd.utils.params import FlatParams
    ps = [("a", torch.nn.Parameter(torch.randn(4000))), ("b", torch.nn.Parameter(torch.randn(3000)))]
    flat = FlatParams(ps, "cpu", shadow=False)
    dp = DataParallel(flat, bucket_mb=0.01)
    dp.begin_step()
    s = flat.slots[0]
    bi = dp.param_bucket[id(s.param)]
    before = list(dp._pending)
    monkeypatch.setattr(torch.cuda, "is_available", lambda: True)
    monkeypatch.setattr(torch.cuda, "is_current_stream_capturing", lambda: True)
    dp._on_ready(s.param)
    assert dp._pending == before and not any(dp._launched)
    monkeypatch.setattr(torch.cuda, "is_current_stream_capturing", lambda: False)
    dp._on_ready(s.param)
    assert dp._pending[bi] == before[bi] - 1


def _worker_ddp_accum_hooks(rank, world, port, q):
    """grad_ready fires per micro-batch (via the ops' _sink); with accum=2 the overlapped buckets
    must reduce only after the last micro-batch, and a param announced twice counts once."""
    _init(rank, world, port)
    from mobilefinetuner_amd.ops import functional as Fx
    from mobilefinetuner_amd.parallel.ddp import DataParallel
    from mobilefinetuner_amd.utils.params import FlatParams
    ps = [(f"p{i}", torch.nn.Parameter(torch.zeros(3000 + 100 * i))) for i in range(4)]
    flat = FlatParams(ps, "cpu", shadow=False)
    dp = DataParallel(flat, bucket_mb=0.01)
    assert len(dp.buckets) > 1 and dp._hook is not None
    dp.begin_step()
    flat.grad.zero_()
    gen = torch.Generator().manual_seed(100 + rank)
    total = torch.zeros_like(flat.grad)
    for micro in range(2):
        dp.last_micro = micro == 1
        for sl in flat.slots:
            p = sl.param
            g = torch.randn(p.shape, generator=gen)
            total[sl.offset:sl.offset + sl.numel] += g
            Fx._sink(p, g)  # accumulates into p.grad and calls grad_ready(p)
            if micro == 1:
                Fx.grad_ready(p)  # a second announcement (tied weights) must not double count
    dp.finish()
    q.put((rank, flat.grad.clone().numpy(), total.clone().numpy()))
    dist.destroy_process_group()


def test_ddp_overlap_with_grad_accumulation():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker_ddp_accum_hooks, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    out = dict((r, (torch.as_tensor(g), torch.as_tensor(t))) for r, g, t in [q.get(timeout=300) for _ in ps])
    for p in ps:
        p.join(60)
    want = (out[0][1] + out[1][1]) / 2  # mean over ranks of the summed micro-batch grads
    assert torch.allclose(out[0][0], want, atol=1e-6) and torch.allclose(out[1][0], want, atol=1e-6)


def _worker_bucketed_reduce(rank, world, port, q, stage, bf16):
    """Hook-driven bucketed reduction: ZeRO-2 reduces every bucket segment to its owner (the owned
    shard must equal the rank mean), DDP/ZeRO-1 all-reduce; optionally through a bf16 comm buffer."""
    _init(rank, world, port)
    from mobilefinetuner_amd.ops import functional as Fx
    from mobilefinetuner_amd.parallel.ddp import DataParallel
    from mobilefinetuner_amd.utils.params import FlatParams
    ps = [(f"p{i}", torch.nn.Parameter(torch.zeros(2000 + 333 * i))) for i in range(5)]
    flat = FlatParams(ps, "cpu", shadow=False, pad_multiple=world)
    shard = flat.numel // world if stage == 2 else None
    dp = DataParallel(flat, bucket_mb=0.01, broadcast_from=None, shard=shard,
                      reduce_dtype=torch.bfloat16 if bf16 else None)
    assert len(dp.buckets) > 1 and dp._hook is not None
    # the buckets tile the buffer exactly
    spans = sorted((b["lo"], b["hi"]) for b in dp.buckets)
    assert spans[0][0] == 0 and spans[-1][1] == flat.numel and all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
    dp.begin_step()
    flat.grad.zero_()
    gen = torch.Generator().manual_seed(7 + rank)
    local = torch.zeros_like(flat.grad)
    for sl in reversed(flat.slots):
        g = torch.randn(sl.param.shape, generator=gen)
        local[sl.offset:sl.offset + sl.numel] = g
        Fx._sink(sl.param, g)
    dp.finish()
    lo, hi = dp.owned()
    q.put((rank, lo, hi, flat.grad.clone().numpy(), local.numpy() if torch.is_tensor(local) else local))
    dp.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("stage,bf16", [(2, False), (2, True), (0, True)])
def test_bucketed_reduce_owner_and_bf16(stage, bf16):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker_bucketed_reduce, args=(r, 2, port, q, stage, bf16)) for r in range(2)]
    for p in ps:
        p.start()
    out = {r: (lo, hi, torch.as_tensor(g), torch.as_tensor(l)) for r, lo, hi, g, l in [q.get(timeout=300) for _ in ps]}
    for p in ps:
        p.join(60)
    want = (out[0][3] + out[1][3]) / 2
    tol = 2e-2 if bf16 else 1e-6
    covered = 0
    for r, (lo, hi, g, _) in out.items():
        assert torch.allclose(g[lo:hi], want[lo:hi], atol=tol), (r, (g[lo:hi] - want[lo:hi]).abs().max())
        covered += hi - lo
    assert covered == (want.numel() if stage == 2 else 2 * want.numel())


def _worker_zero_nonfinite(rank, world, port, q):
    """A NaN in the shard of ONE rank: every rank must skip the step, and the applied-step counter
    (bias correction) must not advance."""
    _init(rank, world, port)
    from mobilefinetuner_amd.parallel.zero import ZeroOptimizer
    from mobilefinetuner_amd.utils.params import FlatParams
    ps = [("w", torch.nn.Parameter(torch.ones(4096)))]
    flat = FlatParams(ps, "cpu", shadow=False, pad_multiple=world)
    opt = ZeroOptimizer(flat, 2, lr=1e-2, weight_decay=0.0, max_grad_norm=1.0)
    flat.grad.fill_(0.1)
    opt.reduce_gradients()
    opt.step()
    after1 = flat.master.clone()
    flat.grad.fill_(0.1)
    if rank == 1:
        flat.grad[flat.numel - 5] = float("nan")  # lands in rank 1's shard only
    opt.reduce_gradients()
    opt.step()
    opt.gather_master()
    q.put((rank, torch.equal(after1, flat.master), opt.step_count, int(opt.skipped_dev.item())))
    dist.destroy_process_group()


def test_zero_nonfinite_skip_is_global():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker_zero_nonfinite, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    out = dict((r, rest) for r, *rest in [q.get(timeout=300) for _ in ps])
    for p in ps:
        p.join(60)
    for r in (0, 1):
        unchanged, steps, skipped = out[r]
        assert unchanged, f"rank {r} applied a step the other rank skipped"
        assert steps == 1 and skipped == 1


def _worker_zero_save(rank, world, port, path, q):
    _init(rank, world, port)
    from mobilefinetuner_amd.data.wikitext2 import LMDataset, WT2Config
    from mobilefinetuner_amd.io import safetensors as st
    from mobilefinetuner_amd.models.gpt2 import GPT2Config, GPT2Model
    from mobilefinetuner_amd.train.trainer import TrainConfig, Trainer
    from mobilefinetuner_amd.utils.params import FlatParams
    m = GPT2Model(GPT2Config.preset("gpt2-tiny"), dtype=torch.float32, device="cpu", seed=11)
    m.set_full_finetune()
    flat = FlatParams(m.named_parameters(), "cpu", shadow=True, pad_multiple=world)
    toks = torch.randint(0, 1000, (8000,), generator=torch.Generator().manual_seed(0), dtype=torch.int64).int()
    ds = LMDataset(WT2Config(seq_len=32, seed=1, rank=rank, world=world), "train", toks)
    tc = TrainConfig(steps=3, batch_size=2, lr=1e-3, log_interval=1, use_graph=False)
    tr = Trainer(m, flat, ds, None, tc, torch.device("cpu"), zero_stage=2)
    tr.train()
    tr.save_state(path)
    tr.opt.gather_master()
    full = {n: p.detach().clone() for n, p in m.named_parameters()}
    dist.barrier()
    saved = st.load_file(os.path.join(path, "trainable.safetensors"))
    ok = all(torch.equal(saved[n].float(), full[n].float()) for n in full)
    q.put((rank, ok))
    dist.destroy_process_group()


def test_zero2_checkpoint_has_every_shard(tmp_path):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker_zero_save, args=(r, 2, port, str(tmp_path), q)) for r in range(2)]
    for p in ps:
        p.start()
    out = dict(q.get(timeout=600) for _ in ps)
    for p in ps:
        p.join(60)
    assert out[0] and out[1]


def test_bench_spawns_ranks_cpu_smoke():
    """bench.py --gpus 2 without a launcher spawns 2 rank processes itself (no re-exec) and reports
    the launched world size: 2 ranks (gloo) on no GPU -- n_gpus counts physical devices."""
    import json
    import subprocess
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
                        "--cpu_smoke"], capture_output=True, text=True, timeout=600,
                       env={k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")})
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 0 and out["config"]["ranks"] == 2 and out["config"]["backend"] == "gloo"
    assert out["config"]["parallelism"] == "dp2"
    assert out["config"]["global_batch"] == 2 * out["config"]["micro_batch_per_gpu"]
