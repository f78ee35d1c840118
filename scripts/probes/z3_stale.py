"""Locate the element a ZeRO-3 + host-offload DP run leaves at its initial value (tests/test_engine_dist_gpu.py
test_native_dp_two_ranks_match_single_process[extra8]): run the same three CLI invocations and print it."""
import os
import sys
import tempfile

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "tests"))
import test_engine_dist_gpu as T  # noqa: E402
from native_logs import loss_list  # noqa: E402
from mobilefinetuner_amd.io import safetensors as st  # noqa: E402

extra = sys.argv[1:] or ["--zero_stage", "3", "--offload", "host"]
tmp = tempfile.mkdtemp()
ref_out, dp_out, init_out = (os.path.join(tmp, n) for n in ("ref.safetensors", "dp.safetensors", "init.safetensors"))
ref = T._single("gpt2_full_finetune", T.FULL + ["--output_path", ref_out], "--batch_size", 8)
res = T._run_ranks([T._bin("gpt2_full_finetune"), *T.FULL, "--batch_size", "4", "--output_path", dp_out, *extra], 2)
print("rcs", [r[0] for r in res], "losses ref", loss_list(ref.stdout, True), "dp", loss_list(res[0][1], True))
T._single("gpt2_full_finetune", [x for x in T.FULL if x not in ("--steps", "6")] + ["--steps", "0", "--output_path", init_out],
          "--batch_size", 8)
a, b, w0 = st.load_file(ref_out), st.load_file(dp_out), st.load_file(init_out)
for k in a:
    moved = a[k] != w0[k]
    stale = moved & (b[k] == w0[k])
    if stale.any():
        idx = stale.nonzero()
        print(k, tuple(a[k].shape), "stale", idx[:5].tolist(), "w0", w0[k][stale][:5].tolist(), "ref", a[k][stale][:5].tolist())
print("done")
for name, t in (("ref", a), ("dp", b)):
    tot = sum(v.numel() for v in t.values())
    bfv = sum(int((v.float().view(torch.int32) & 0xFFFF == 0).sum()) for v in t.values())
    print(name, "dtype", next(iter(t.values())).dtype, "bf16-representable fraction", bfv / tot)
print("per tensor: max|ref-dp|, max|ref-w0|, median |ref-dp|/|ref-w0|")
for k in a:
    d = (a[k].float() - b[k].float()).abs()
    m = (a[k].float() - w0[k].float()).abs()
    r = (d / m.clamp(min=1e-12))
    print(f"  {k:28s} {d.max().item():.3e} {m.max().item():.3e} {r.median().item():.3e}")
