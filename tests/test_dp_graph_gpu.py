"""Data-parallel reducers with the hipGraph step, on one GPU with a 1-rank RCCL group
(MFT_DP_FORCE_COMM=1 keeps the collectives even though there is nothing to average): the bucketed
all-reduce (DDP), its bf16 variant and the ZeRO-2 per-bucket reduce-scatter, both recorded into the
graph from the backward's grad-ready hooks (MFT_GRAPH_COMM=1, the default) and run after each
replay (MFT_GRAPH_COMM=0), while RCCL's watchdog polls during the capture; the replayed steps equal
the no-DP step."""
import os

import pytest
import torch
import torch.distributed as dist

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module")
def rccl1():
    os.environ["MFT_DP_FORCE_COMM"] = "1"
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", str(29700 + os.getpid() % 1000))
    created = not dist.is_initialized()
    if created:
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    yield
    os.environ.pop("MFT_DP_FORCE_COMM", None)
    if created:
        dist.destroy_process_group()


def _run(kind, steps=6, graph_comm=False):
    from mobilefinetuner_amd.models.gpt2 import GPT2Config, GPT2Model
    from mobilefinetuner_amd.optim.adamw import FusedAdamW
    from mobilefinetuner_amd.parallel.ddp import DataParallel
    from mobilefinetuner_amd.parallel.zero import ZeroOptimizer, ZeroReducer
    from mobilefinetuner_amd.train.engine import TrainStep
    from mobilefinetuner_amd.utils.params import FlatParams

    m = GPT2Model(GPT2Config.preset("gpt2-tiny"), device=DEV, seed=5)
    m.set_full_finetune()
    flat = FlatParams(m.named_parameters(), DEV)
    kw = dict(lr=1e-3, weight_decay=0.01, max_grad_norm=1.0)
    if kind == "zero2":
        opt = ZeroOptimizer(flat, 2, bucket_mb=0.25, **kw)
        dp = ZeroReducer(opt)
    else:
        opt = FusedAdamW(flat, **kw)
        dp = None if kind == "none" else DataParallel(flat, bucket_mb=0.25, broadcast_from=None,
                                                      reduce_dtype=torch.bfloat16 if kind == "bf16" else None)
    st = TrainStep(m, flat, opt, dp=dp, use_graph=True)
    ids = torch.randint(0, 1000, (8, 65), device=DEV, generator=torch.Generator(device=DEV).manual_seed(2))
    b = [(ids[:, :-1].contiguous(), ids[:, 1:].contiguous())]
    losses = [float(st(b).item()) for _ in range(steps)]
    w = flat.master.clone()
    if dp is not None:
        nb = len(dp.zero.reducer.buckets) if kind == "zero2" else len(dp.buckets)
        assert nb > 1 and st.graph_comm == graph_comm, (kind, nb)
        dp.close()
    return losses, w


MODES = [False, True]  # eager reduction after the replay / collectives recorded into the graph (default)


@pytest.mark.parametrize("graph_comm", MODES)
@pytest.mark.parametrize("kind", ["ddp", "bf16", "zero2"])
def test_reducer_with_graph_step_matches_no_dp(rccl1, kind, graph_comm, monkeypatch):
    """(deterministic reductions: the embedding's scatter-add otherwise differs in the last bits
    between two runs, and AdamW's per-element normalisation turns such noise on near-zero gradients
    into +-lr updates within a few steps.  ZeRO-2 also sums the grad-norm^2 over its bucket-ordered
    chunks -- a different fp32 order than the flat buffer's -- hence its looser weight bound.)"""
    from mobilefinetuner_amd.ops import functional as Fx
    monkeypatch.setenv("MFT_GRAPH_COMM", "1" if graph_comm else "0")
    Fx.set_deterministic(True)
    try:
        ref_l, ref_w = _run("none")
        l, w = _run(kind, graph_comm=graph_comm)
    finally:
        Fx.set_deterministic(False)
    tol = 3e-2 if kind == "bf16" else 2e-3
    assert l == pytest.approx(ref_l, rel=tol, abs=tol), (kind, l, ref_l)
    err = ((w - ref_w).norm() / ref_w.norm()).item()
    assert err < {"bf16": 5e-3, "zero2": 2e-3}.get(kind, 1e-4), (kind, err)
