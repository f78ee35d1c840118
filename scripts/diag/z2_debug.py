"""ZeRO-2 (chunked reduce-scatter) vs plain AdamW on one GPU, 1-rank RCCL: per-step weight diffs,
eager and graph-captured, with and without the backward-overlapped hooks."""
import os
import sys

import torch
import torch.distributed as dist

os.environ.update(MFT_DP_FORCE_COMM="1", MASTER_ADDR="127.0.0.1", MASTER_PORT="29733")
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
from mobilefinetuner_amd.models.gpt2 import GPT2Config, GPT2Model  # noqa: E402
from mobilefinetuner_amd.optim.adamw import FusedAdamW  # noqa: E402
from mobilefinetuner_amd.parallel.zero import ZeroOptimizer, ZeroReducer  # noqa: E402
from mobilefinetuner_amd.train.engine import TrainStep  # noqa: E402
from mobilefinetuner_amd.utils.params import FlatParams  # noqa: E402


SNAP = []
_orig_step = ZeroOptimizer.step


def _snap_step(self, sumsq_ready=False):
    torch.cuda.synchronize()
    SNAP.append((self.reducer.own_grad.clone(), self.flat.grad.clone()))
    return _orig_step(self, sumsq_ready)


ZeroOptimizer.step = _snap_step
from mobilefinetuner_amd.parallel.ddp import DataParallel  # noqa: E402
_orig_finish = DataParallel.finish
SYNC = [False]


def _finish(self):
    if SYNC[0]:
        torch.cuda.synchronize()
    return _orig_finish(self)


DataParallel.finish = _finish


def run(kind, graph, overlap, steps=5):
    m = GPT2Model(GPT2Config.preset("gpt2-tiny"), device="cuda", seed=5)
    m.set_full_finetune()
    flat = FlatParams(m.named_parameters(), "cuda")
    kw = dict(lr=1e-3, weight_decay=0.01, max_grad_norm=1.0)
    if kind == "zero2":
        opt = ZeroOptimizer(flat, 2, bucket_mb=0.25, overlap=overlap, **kw)
        dp = ZeroReducer(opt)
    else:
        opt, dp = FusedAdamW(flat, **kw), None
    st = TrainStep(m, flat, opt, dp=dp, use_graph=graph)
    ids = torch.randint(0, 1000, (8, 65), device="cuda", generator=torch.Generator(device="cuda").manual_seed(2))
    b = [(ids[:, :-1].contiguous(), ids[:, 1:].contiguous())]
    ws, gs = [], []
    for _ in range(steps):
        st(b)
        torch.cuda.synchronize()
        ws.append(flat.master.clone())
        gs.append((opt.reducer.own_grad.clone() if kind == "zero2" else None, flat.grad.clone(), flat.shadow.clone()))
    global flat_slots
    flat_slots = flat.slots
    return ws, gs, opt


x = torch.randn(1 << 20, device="cuda")
for op in (dist.ReduceOp.AVG, dist.ReduceOp.SUM):
    out = torch.empty_like(x)
    dist.reduce_scatter_tensor(out, x, op=op)
    torch.cuda.synchronize()
    print("1-rank RCCL reduce_scatter", op, "max |out - x| =", (out - x).abs().max().item(), flush=True)
    y = x[4096:8192]
    out2 = torch.empty_like(y)
    dist.reduce_scatter_tensor(out2, y, op=op)
    torch.cuda.synchronize()
    print("  offset slice: max |out - x| =", (out2 - y).abs().max().item(), flush=True)
flat_slots = []
for sync in (False,):
  SYNC[0] = sync
  print("sync before finish:", sync, flush=True)
  for graph in (False,):
    for overlap in (False,):
        w0, g0, _ = run("none", graph, overlap)
        w1, g1, opt = run("zero2", graph, overlap)
        R = opt.reducer
        diffs = [((a - b).norm() / a.norm()).item() for a, b in zip(w0, w1)]
        # the reduced chunk vs the plain grad, per step
        gd = []
        for (own, fg, _), (_, fg0, _) in zip(g1, g0):
            full = torch.cat([fg0[b_["lo"]:b_["hi"]] for b_ in R.buckets])
            gd.append(((own - full).norm() / full.norm()).item())
        fgd = [((fg0 - fg).norm() / fg0.norm()).item() for (_, fg, _), (_, fg0, _) in zip(g1, g0)]
        shd = []
        for (_, _, s1), (_, _, s0) in zip(g1, g0):
            d = (s1.float() - s0.float()).abs()
            nz = torch.nonzero(d > 0).flatten()
            who = []
            if nz.numel():
                j = int(nz[0])
                who = [(sl.name, j - sl.offset) for sl in flat_slots if sl.offset <= j < sl.offset + sl.numel]
            shd.append((int((d > 0).sum()), who))
        print("shadow mismatches per step (count, first):", shd, flush=True)
        own, fgz = SNAP[0]
        bad = []
        for i, b_ in enumerate(R.buckets):
            o, c = R.own_off[i], b_["c"]
            dd = (own[o:o + c] - fgz[b_["lo"]:b_["hi"]]).abs()
            d = dd.max().item()
            if d > 0:
                j = int(dd.argmax()) + b_["lo"]
                who = [(sl.name, j - sl.offset) for sl in b_["slots"] if sl.offset <= j < sl.offset + sl.numel]
                nbad = int((dd > 0).sum())
                bad.append((i, d, nbad, who))
        print("pre-step own vs flat.grad mismatching buckets:", len(bad), "of", len(R.buckets), bad[:6], flush=True)
        SNAP.clear()
        print("flat.grad rel diff per step", ['%.1e' % d for d in fgd])
        print(f"graph={graph} overlap={overlap}: weight rel diff per step {['%.1e' % d for d in diffs]}  "
              f"grad rel diff {['%.1e' % d for d in gd]}", flush=True)
dist.destroy_process_group()
sys.exit(0)
