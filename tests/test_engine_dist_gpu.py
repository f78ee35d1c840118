"""Native data parallelism (libmft engine/comm.h + engine/dist.h) with several ranks on ONE GPU.

The loopback backend (MFT_COMM_BACKEND=loopback: host TCP star, collectives as D2H copy -> host
reduce -> H2D copy, recorded into the hipGraph as host nodes) lets N native rank processes share a
single MI355X -- RCCL refuses two ranks on one device -- so the multi-rank code paths run here:
rank-0 weight broadcast, per-rank data shards, bucketed gradient reduction from the grad-ready hooks,
ZeRO-1 / ZeRO-2 partitioned AdamW (+ pinned-host moments), the bf16 shadow all-gather, reduced losses
and eval sums.  Each is checked against ONE process at the same GLOBAL batch (--deterministic).
RCCL itself is exercised on a 1-rank group with the whole ZeRO-2 step (reduce-scatter, all-gather)
recorded into the hipGraph.  Failure detection: a rank that dies makes its peer exit non-zero.
"""
import os
import re
import socket
import subprocess
import time

import pytest
import torch
from native_logs import PLOT_PATTERN1, PLOT_PATTERN2, loss_list

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "mobilefinetuner_amd", "bin")


def _bin(name):
    p = os.path.join(BIN, name)
    if not os.path.exists(p):
        pytest.fail(f"{p} missing: run python -m mobilefinetuner_amd._build")
    return p


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _env(rank=0, world=1, port=None, backend="loopback", **extra):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MFT_DP_FORCE_COMM"):
        env.pop(k, None)
    if world > 1 or extra.get("MFT_DP_FORCE_COMM") == "1":
        env.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port or _port()), MFT_COMM_BACKEND=backend)
    env.update({k: str(v) for k, v in extra.items()})
    return env


def _run_ranks(cmd, world, timeout=150, backend="loopback", extra_env=None, per_rank=None):
    """Start `world` native rank processes (one shared GPU); returns [(rc, stdout, stderr)].  A rank still
    running after `timeout` s (these runs take seconds) fails the test with every rank's output tail --
    well inside the GPU runner's 180-s silence limit."""
    port = _port()
    procs = []
    for r in range(world):
        c = cmd + (per_rank(r) if per_rank else [])
        procs.append(subprocess.Popen(c, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                                      env=_env(r, world, port, backend, **(extra_env or {}))))
    out = []
    for p in procs:
        try:
            o, e = p.communicate(timeout=timeout)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            tails = []
            for r, q in enumerate(procs):
                o, e = q.communicate()
                tails.append(f"--- rank {r} (rc {q.returncode}) stdout ---\n{(o or '')[-1500:]}\n"
                             f"--- rank {r} stderr ---\n{(e or '')[-1500:]}")
            raise AssertionError(f"{world} ranks timed out after {timeout} s: {' '.join(cmd)}\n" + "\n".join(tails))
        out.append((p.returncode, o, e))
    return out


FULL = ["--random_init", "--model", "gpt2-tiny", "--synthetic_data", "--synthetic_tokens", "100000", "--seq_len", "64",
        "--lr", "1e-3", "--log_interval", "1", "--deterministic", "--steps", "6", "--bucket_mb", "0.25"]


def _single(prog, args, batch_flag, batch):
    r = subprocess.run([_bin(prog), *args, batch_flag, str(batch)], capture_output=True, text=True, timeout=150,
                       env=_env())
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    return r


@pytest.mark.parametrize("extra,tol", [
    ([], 2e-4),
    (["--zero_stage", "1"], 2e-4),
    (["--zero_stage", "2"], 2e-4),
    (["--zero_stage", "2", "--offload", "host"], 3e-3),   # bf16 stochastically-rounded moments
    (["--bf16_grads"], 1e-2),
    (["--zero_stage", "2", "--no_overlap", "--no_graph"], 2e-4),
    (["--zero_stage", "3"], 2e-4),
    (["--zero_stage", "3", "--no_graph", "--grad_accum_steps", "1"], 2e-4),
    (["--zero_stage", "3", "--offload", "host"], 3e-3),
    (["--zero_stage", "2", "--offload", "host", "--offload_moments", "fp32"], 2e-4),  # fp32 host moments: exact
    (["--zero_stage", "3", "--offload", "host", "--offload_moments", "fp32"], 2e-4),  # streamed (default)
    (["--zero_stage", "3", "--offload", "host", "--offload_mode", "zerocopy"], 3e-3),
    (["--zero_stage", "2", "--offload", "disk", "--offload_moments", "fp32"], 2e-4),  # moments in files, streamed
])
def test_native_dp_two_ranks_match_single_process(tmp_path, extra, tol):
    """2 loopback ranks x batch 4 == 1 process x batch 8 (GPT-2-tiny full fine-tune, ~8 buckets):
    the same per-step losses and the same final weights."""
    if "disk" in extra:
        extra = extra + ["--offload_dir", str(tmp_path / "offload")]
    ref_out = str(tmp_path / "ref.safetensors")
    ref = _single("gpt2_full_finetune", FULL + ["--output_path", ref_out], "--batch_size", 8)
    want = loss_list(ref.stdout, True)
    dp_out = str(tmp_path / "dp.safetensors")
    res = _run_ranks([_bin("gpt2_full_finetune"), *FULL, "--batch_size", "4", "--output_path", dp_out, *extra], 2)
    for rc, o, e in res:
        assert rc == 0, o[-2000:] + e[-2000:]
    out0 = res[0][1]
    assert "data parallel: rank 0 of 2 (loopback" in out0, out0[:3000]
    z3 = "3" in extra[1:2]
    assert ("ZeRO-3 over 2 rank(s)" if z3 else "bucket(s)") in out0, out0[:3000]
    got = loss_list(out0, True)
    assert len(got) == 6 and got == pytest.approx(want, rel=tol, abs=tol), (extra, got, want)
    from mobilefinetuner_amd.io import safetensors as st
    # the final weights agree, and no element the reference updated stayed EXACTLY at its initial
    # value in the DP export (weight decay moves every updated element): a chunk a rank never updated
    # or exported stale, or LayerNorm values a non-owning rank kept stale (fp32-compute
    # parameters under ZeRO-1/2), fail here.  (Elementwise update deltas cannot be compared tightly:
    # parameters with a ~0 true gradient, e.g. the key bias, get noise-driven Adam steps -- and such an
    # element may legitimately end exactly where it started in one run and not the other: bf16 moments
    # measured one wte element the reference moved by 2.4e-6 in total (vs ~3.7e-3 for the tensor) left at
    # its initial value, scripts/probes/z3_stale.py.  "Moved" therefore means moved by more than 1e-5.)
    init_out = str(tmp_path / "init.safetensors")
    _single("gpt2_full_finetune", [x for x in FULL if x not in ("--steps", "6")] + ["--steps", "0", "--output_path",
                                                                                       init_out], "--batch_size", 8)
    a, b, w0 = st.load_file(ref_out), st.load_file(dp_out), st.load_file(init_out)
    wtol = 50 * tol
    for k in a:
        assert torch.allclose(a[k], b[k], atol=wtol, rtol=wtol), (extra, k, (a[k] - b[k]).abs().max())
        moved = (a[k] - w0[k]).abs() > 1e-5
        stale = moved & (b[k] == w0[k])
        assert moved.any() and int(stale.sum()) == 0, (extra, k, int(stale.sum()), int(moved.sum()))


@pytest.mark.parametrize("moments,chunk", [("fp32", ""), ("fp32", "1000"), ("bf16", "1000")])
def test_native_offload_disk_matches_device_moments(tmp_path, moments, chunk):
    """--offload disk (AdamW moments in file mappings, streamed through device chunks each step; eager)
    == moments on the device (fp32) / in pinned host DRAM (bf16, the same stochastic rounding): the same
    per-step losses and final weights, several chunks per step (MFT_DISK_CHUNK), and the moment files on disk."""
    import os
    env_chunk = {"MFT_DISK_CHUNK": chunk} if chunk else {}
    ref_args = ["--offload", "host", "--offload_moments", "bf16"] if moments == "bf16" else []
    ref_out, out = str(tmp_path / "ref.safetensors"), str(tmp_path / "disk.safetensors")
    ref = _single("gpt2_full_finetune", FULL + ["--output_path", ref_out] + ref_args, "--batch_size", 4)
    d = str(tmp_path / "offload")
    r = subprocess.run([_bin("gpt2_full_finetune"), *FULL, "--batch_size", "4", "--output_path", out, "--offload", "disk",
                        "--offload_dir", d, "--offload_moments", moments], capture_output=True, text=True, timeout=150,
                       env=_env(**env_chunk))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "AdamW moments on disk" in r.stdout and "step runs eagerly" in r.stdout, r.stdout[:3000]
    got, want = loss_list(r.stdout, True), loss_list(ref.stdout, True)
    assert len(got) == 6 and got == pytest.approx(want, rel=1e-5, abs=1e-5), (got, want)
    from mobilefinetuner_amd.io import safetensors as st
    a, b = st.load_file(ref_out), st.load_file(out)
    for k in a:
        assert torch.allclose(a[k], b[k], atol=1e-5, rtol=1e-5), (k, (a[k] - b[k]).abs().max())
    for name in ("m", "v"):
        f = os.path.join(d, f"adamw_{name}.rank0.bin")
        assert os.path.getsize(f) > 0 and any(open(f, "rb").read(1 << 16)), f  # written back, not all zero


def test_native_dp_lora_and_gemma_two_ranks():
    """LoRA (one fused bucket) on GPT-2-tiny and Gemma-3-tiny: 2 loopback ranks == 1 process."""
    lora = ["--random_init", "--model", "gpt2-tiny", "--synthetic_data", "--synthetic_tokens", "100000", "--seq_len",
            "64", "--lr", "1e-3", "--log_interval", "1", "--deterministic", "--steps", "5"]
    want = loss_list(_single("gpt2_lora_finetune", lora, "--batch_size", 8).stdout, True)
    res = _run_ranks([_bin("gpt2_lora_finetune"), *lora, "--batch_size", "4"], 2)
    assert all(rc == 0 for rc, _, _ in res), res[0][1][-2000:] + res[0][2][-2000:]
    assert loss_list(res[0][1], True) == pytest.approx(want, rel=2e-4, abs=2e-4)
    gem = ["--random_init", "--model", "gemma3-tiny", "--synthetic_data", "--synthetic_tokens", "100000", "--seq_len",
           "64", "--lr", "1e-3", "--log_interval", "1", "--deterministic", "--max_steps", "5", "--lora_dropout", "0",
           "--lr_schedule", "constant", "--zero_stage", "1"]
    want = loss_list(_single("train_lora_gemma", gem[:-2], "--batch", 8).stdout, True)
    res = _run_ranks([_bin("train_lora_gemma"), *gem, "--batch", "4"], 2)
    assert all(rc == 0 for rc, _, _ in res), res[0][1][-2000:] + res[0][2][-2000:]
    assert loss_list(res[0][1], True) == pytest.approx(want, rel=2e-4, abs=2e-4)


def test_native_rccl_zero2_step_in_graph():
    """A 1-rank RCCL group running ZeRO-2 with the whole step (bucket reduce-scatters on the comm
    stream, partitioned AdamW with the all-reduced norm, shadow all-gather) recorded into ONE
    hipGraph: the capture succeeds and the losses match the plain single-process step."""
    want = loss_list(_single("gpt2_full_finetune", FULL, "--batch_size", 4).stdout, True)
    r = subprocess.run([_bin("gpt2_full_finetune"), *FULL, "--batch_size", "4", "--zero_stage", "2"],
                       capture_output=True, text=True, timeout=150, env=_env(backend="rccl", MFT_DP_FORCE_COMM="1"))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "data parallel: rank 0 of 1 (rccl" in r.stdout and "ZeRO-2" in r.stdout, r.stdout[:3000]
    assert loss_list(r.stdout, True) == pytest.approx(want, rel=2e-4, abs=2e-4)


def test_native_rccl_zero3_step_in_graph():
    """ZeRO-3 on a 1-rank RCCL group: per-block all-gathers into the two device slots, per-block
    gradient reduce-scatters and the partitioned AdamW, all recorded into ONE hipGraph, with the
    plain single-process losses (2 micro-batches: the reduce-scatters accumulate)."""
    args = FULL + ["--batch_size", "2", "--grad_accum_steps", "2"]
    want = loss_list(_single("gpt2_full_finetune", args[:-2], "--grad_accum_steps", 2).stdout, True)
    r = subprocess.run([_bin("gpt2_full_finetune"), *args, "--zero_stage", "3"],
                       capture_output=True, text=True, timeout=150, env=_env(backend="rccl", MFT_DP_FORCE_COMM="1"))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "ZeRO-3 over 1 rank(s) [rccl]" in r.stdout and "hipGraph" in r.stdout, r.stdout[:3000]
    assert loss_list(r.stdout, True) == pytest.approx(want, rel=2e-4, abs=2e-4)


@pytest.mark.parametrize("every", [1, 2])
def test_native_zero3_streamed_optimizer_flushes_in_graph_mode(tmp_path, every):
    """the host-streamed ZeRO-3 AdamW (update applied per unit during the NEXT forward)
    issues its gated updates from device state, not from a host flag a hipGraph replay never advances.
    With an eval every step (a flush after every replay) or every 2 steps (a flush before the step-3
    capture), two loopback ranks in graph mode must end with the same weights and losses as the
    eager run without evaluations."""
    base = FULL + ["--batch_size", "4", "--zero_stage", "3", "--offload", "host", "--offload_moments", "fp32"]
    ref_out, out = str(tmp_path / "eager.safetensors"), str(tmp_path / "graph.safetensors")
    inplace = {"MFT_Z3_STAGED": "0"}  # (the staged variant runs eagerly: test_native_zero3_staged_moments_match_in_place)
    ref = _run_ranks([_bin("gpt2_full_finetune"), *base, "--no_graph", "--output_path", ref_out], 2, extra_env=inplace)
    assert all(rc == 0 for rc, _, _ in ref), ref[0][1][-2000:] + ref[0][2][-2000:]
    got = _run_ranks([_bin("gpt2_full_finetune"), *base, "--eval_interval", str(every), "--eval_batches", "2",
                      "--output_path", out], 2, extra_env=inplace)
    assert all(rc == 0 for rc, _, _ in got), got[0][1][-2000:] + got[0][2][-2000:]
    assert "hipGraph" in got[0][1], got[0][1][:3000]
    assert loss_list(got[0][1], True) == pytest.approx(loss_list(ref[0][1], True), rel=2e-4, abs=2e-4)
    from mobilefinetuner_amd.io import safetensors as st
    a, b = st.load_file(ref_out), st.load_file(out)
    # (--deterministic: graph and eager run the same kernels in the same order; one missing or late
    # Adam step would move elements by ~lr = 1e-3)
    for k in a:
        assert torch.allclose(a[k], b[k], atol=2e-5, rtol=0), (every, k, (a[k] - b[k]).abs().max())


@pytest.mark.parametrize("slots,moments,capture", [("1", "fp32", ""), ("2", "bf16", ""), ("", "bf16", ""), ("", "bf16", "1"),
                                                   ("1", "fp32", "1")])
def test_native_zero3_staged_moments_match_in_place(tmp_path, slots, moments, capture):
    """The staged host-moment optimizer (device slots refilled by SDMA copies on one copy stream: the slot
    written back after its update and prefetched for its next user, across the step boundary) ends with the
    same weights as the in-place zero-copy update (MFT_Z3_STAGED=0, eager), two loopback ranks, evaluations
    (flushes) every 2 steps -- with one slot (every update waits for its own prefetch), two, and the
    default; eager (the default: faster for this step) and captured in a hipGraph (MFT_Z3_CAPTURE=1, since
    the round-6 fix of the communication stream's self-wait)."""
    base = FULL + ["--batch_size", "4", "--zero_stage", "3", "--offload", "host", "--offload_moments", moments]
    ref_out, out = str(tmp_path / "inplace.safetensors"), str(tmp_path / "staged.safetensors")
    ref = _run_ranks([_bin("gpt2_full_finetune"), *base, "--no_graph", "--output_path", ref_out], 2,
                     extra_env={"MFT_Z3_STAGED": "0"})
    assert all(rc == 0 for rc, _, _ in ref), ref[0][1][-2000:] + ref[0][2][-2000:]
    env = {"MFT_Z3_STAGED": "1", **({"MFT_Z3_SLOTS": slots} if slots else {}), **({"MFT_Z3_CAPTURE": capture} if capture else {})}
    got = _run_ranks([_bin("gpt2_full_finetune"), *base, "--eval_interval", "2", "--eval_batches", "2",
                      "--output_path", out], 2, extra_env=env)
    assert all(rc == 0 for rc, _, _ in got), got[0][1][-2000:] + got[0][2][-2000:]
    mode = "hipGraph-captured step" if capture == "1" else "step runs eagerly"
    assert mode in got[0][1] and "slots]" in got[0][1], got[0][1][:3000]
    assert loss_list(got[0][1], True) == pytest.approx(loss_list(ref[0][1], True), rel=2e-4, abs=2e-4)
    from mobilefinetuner_amd.io import safetensors as st
    a, b = st.load_file(ref_out), st.load_file(out)
    for k in a:
        assert torch.allclose(a[k], b[k], atol=2e-5, rtol=0), (slots, k, (a[k] - b[k]).abs().max())


@pytest.mark.parametrize("stage", ["2", "3", "3+offload"])
def test_native_dp_state_resume_two_ranks(tmp_path, stage):
    """ZeRO-2 / ZeRO-3 full-state checkpoint (gathered fp32 master, or each rank's own parameter
    partitions, + one optimizer partition per rank): 4 steps, then both ranks resume from the saved
    state and finish steps 5-8 with the uninterrupted run's losses."""
    extra = ["--offload", "host", "--offload_moments", "fp32"] if stage.endswith("+offload") else []
    base = FULL[:-4] + ["--bucket_mb", "0.25", "--batch_size", "4", "--zero_stage", stage[:1], "--warmup_steps", "100",
                        *extra]
    ref = _run_ranks([_bin("gpt2_full_finetune"), *base, "--steps", "8"], 2)
    assert all(rc == 0 for rc, _, _ in ref)
    want = loss_list(ref[0][1])
    state = str(tmp_path / "state")
    a = _run_ranks([_bin("gpt2_full_finetune"), *base, "--steps", "4", "--state_dir", state], 2)
    assert all(rc == 0 for rc, _, _ in a), a[0][2][-2000:]
    assert os.path.exists(os.path.join(state, "optimizer.rank1.safetensors"))
    b = _run_ranks([_bin("gpt2_full_finetune"), *base, "--steps", "8", "--state_dir", state], 2)
    assert all(rc == 0 for rc, _, _ in b), b[0][2][-2000:]
    assert "resumed full training state" in b[0][1]
    got = loss_list(a[0][1], True) + loss_list(b[0][1], True)
    # (a full fine-tune's last printed digit may differ once across 8 steps: the resumed process
    # runs its first two steps eagerly and captures at step 7; losses are compared to 1e-4)
    assert got == pytest.approx([float(x) for x in want], rel=1e-4, abs=1e-4), (want, got)


def test_native_peer_failure_makes_the_other_rank_exit():
    """rank 1 dies before step 3 (--inject_fault 3:1); rank 0, blocked in that step's
    collective, sees the lost peer and exits with code 3 well within MFT_COMM_TIMEOUT (no hang)."""
    t0 = time.time()
    res = _run_ranks([_bin("gpt2_full_finetune"), *FULL, "--batch_size", "4", "--inject_fault", "3:1"], 2,
                     timeout=120, extra_env={"MFT_COMM_TIMEOUT": "60"})
    dt = time.time() - t0
    (rc0, o0, e0), (rc1, o1, e1) = res
    assert rc1 != 0 and "injected fault at step 3" in e1, e1[-1500:]
    assert rc0 == 3 and "[mft comm] rank 0/2" in e0, (rc0, e0[-2000:])
    assert dt < 100, dt


def test_native_logs_parse_with_the_reference_plotter_regexes():
    """The reference's loss plotter (scripts/Finetune/plot_loss_curve.py:18-19) parses the native
    GPT-2 ([Train] ... step s/S ... loss X) and Gemma ([Step n] Loss=X) console lines."""
    r = _single("gpt2_lora_finetune", FULL[:-4] + ["--steps", "3"], "--batch_size", 4)
    m = [re.search(PLOT_PATTERN2, ln, re.IGNORECASE) for ln in r.stdout.splitlines() if ln.startswith("[Train]")]
    assert len(m) == 3 and all(m), r.stdout[-1500:]
    g = _single("train_lora_gemma", ["--random_init", "--model", "gemma3-tiny", "--synthetic_data", "--synthetic_tokens",
                                     "100000", "--seq_len", "64", "--max_steps", "3", "--log_interval", "1"], "--batch", 4)
    m = [re.search(PLOT_PATTERN1, ln) for ln in g.stdout.splitlines() if ln.startswith("[Step")]
    assert len(m) == 3 and all(m) and [int(x.group(1)) for x in m] == [1, 2, 3], g.stdout[-1500:]


def test_native_bench_json_line(tmp_path):
    """bench.py's default (native engine) path prints the driver's JSON record from the native
    CLI's MFT_BENCH line (a short GPT-2 LoRA run)."""
    import json
    r = subprocess.run(["python", os.path.join(ROOT, "bench.py"), "--steps", "3", "--warmup", "3", "--batch", "64"],
                       capture_output=True, text=True, timeout=160, env=_env(), cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    rec = json.loads(r.stdout.strip().splitlines()[-1])
    assert rec["n_gpus"] == 1 and rec["steps"] == 3 and rec["value"] > 0 and "native" in rec["config"]["engine"]
    assert abs(rec["value"] - 64 * 128 * 3 / (rec["ms_per_step"] * 3 / 1000)) < 0.01 * rec["value"]


def test_native_bench_under_torchrun_two_ranks():
    """The driver's N>1 launch exactly (python -m torch.distributed.run ... bench.py --gpus 2): each
    rank's bench.py starts its native child, the children bootstrap their communicator on
    MASTER_PORT + 1 and rank 0 prints one record for the whole job.  Loopback backend: both ranks
    share the box's one GPU, so the record counts one physical device."""
    import json
    env = _env()
    env["MFT_COMM_BACKEND"] = "loopback"
    r = subprocess.run(["python", "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(_port()),
                        os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "2", "--batch", "64"],
                       capture_output=True, text=True, timeout=160, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    lines = [l for l in r.stdout.strip().splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 1 and rec["config"]["ranks"] == 2 and rec["config"]["global_batch"] == 128
    assert rec["config"]["parallelism"] == "dp2" and rec["steps"] == 3 and rec["value"] > 0
    assert abs(rec["value"] - 2 * 64 * 128 * 3 / (rec["ms_per_step"] * 3 / 1000)) < 0.01 * rec["value"]


@pytest.mark.parametrize("prog,args,bflag", [
    ("gpt2_full_finetune", FULL, "--batch_size"),
    ("gpt2_full_finetune", FULL + ["--zero_stage", "3"], "--batch_size"),
    ("gpt2_lora_finetune", FULL + ["--lora_targets", "AttnQKV,AttnProj,MlpFcIn,MlpFcOut"], "--batch_size"),
    ("train_lora_gemma", ["--random_init", "--model", "gemma3-tiny", "--synthetic_data", "--synthetic_tokens", "100000",
                          "--seq_len", "64", "--lr", "1e-3", "--log_interval", "1", "--deterministic", "--max_steps", "5",
                          "--lora_dropout", "0.1", "--lr_schedule", "constant"], "--batch"),
], ids=["gpt2-full", "gpt2-full-zero3", "gpt2-lora", "gemma-lora-dropout"])
def test_native_activation_checkpointing_same_losses(prog, args, bflag):
    """--activation_checkpointing (autograd.h checkpoint(): each block recomputed in the backward,
    a nested backward through it) trains to the same per-step losses as keeping the activations --
    LoRA dropout masks included (counter-based, identical in the recompute), ZeRO-3 gathers too."""
    want = loss_list(_single(prog, args, bflag, 4).stdout, True)
    extra_env = {"MFT_DP_FORCE_COMM": "1"} if "--zero_stage" in args else {}
    r = subprocess.run([_bin(prog), *args, bflag, "4", "--activation_checkpointing"], capture_output=True, text=True,
                       timeout=150, env=_env(backend="rccl", **extra_env) if extra_env else _env())
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    got = loss_list(r.stdout, True)
    assert len(got) == len(want) and got == pytest.approx(want, rel=1e-5, abs=1e-5), (got, want)


def test_native_two_ranks_print_identical_gemm_choice_maps():
    """Every per-shape GEMM decision is rank-independent: the gemm4 / gemm_s / gemm8 routing is a fixed
    table (no vendor library, no per-process timing), so the two ranks' MFT_GEMM_MAP lines -- kernel per
    shape -- are identical, and none of them names a library GEMM."""
    lora = ["--random_init", "--model", "gpt2-tiny", "--synthetic_data", "--synthetic_tokens", "100000", "--seq_len",
            "64", "--lr", "1e-3", "--log_interval", "1", "--steps", "3", "--batch_size", "4"]
    res = _run_ranks([_bin("gpt2_lora_finetune"), *lora], 2, extra_env={"MFT_GEMM_MAP": "1"})
    assert all(rc == 0 for rc, _, _ in res), res[0][1][-2000:] + res[0][2][-2000:]
    maps = [sorted(l for l in e.splitlines() if l.startswith("[gemm-map]")) for _, _, e in res]
    assert maps[0] and maps[0] == maps[1], (maps[0][:20], maps[1][:20])
    assert not any("hipBLASLt" in l for l in maps[0]), maps[0][:20]
    assert any("gemm_s" in l or "gemm4" in l for l in maps[0]), maps[0][:20]


@pytest.mark.parametrize("extra", [[], ["--zero_stage", "2"], ["--zero_stage", "3"]], ids=["ddp", "zero2", "zero3"])
def test_native_dp_four_ranks_match_single_process(tmp_path, extra):
    """4 loopback ranks x batch 2 == 1 process x batch 8 (GPT-2-tiny full fine-tune): per-step losses and final
    weights, DDP / ZeRO-2 / ZeRO-3 -- so ZeRO-3 == DDP at 4 ranks too.  The bucketed reducers launch every
    bucket's reduction from the backward's grad-ready hooks (overlapped), none from the post-backward sweep."""
    from mobilefinetuner_amd.io import safetensors as st
    ref_out = str(tmp_path / "ref.safetensors")
    want = loss_list(_single("gpt2_full_finetune", FULL + ["--output_path", ref_out], "--batch_size", 8).stdout, True)
    dp_out = str(tmp_path / "dp.safetensors")
    res = _run_ranks([_bin("gpt2_full_finetune"), *FULL, "--batch_size", "2", "--output_path", dp_out, *extra], 4,
                     timeout=160)
    for rc, o, e in res:
        assert rc == 0, o[-2000:] + e[-2000:]
    out0 = res[0][1]
    assert "data parallel: rank 0 of 4 (loopback" in out0, out0[:3000]
    got = loss_list(out0, True)
    assert len(got) == 6 and got == pytest.approx(want, rel=2e-4, abs=2e-4), (extra, got, want)
    if "3" not in extra:
        m = re.search(r"\[dp\] first step: (\d+) of (\d+) bucket", out0)
        assert m and int(m.group(2)) > 1 and m.group(1) == m.group(2), out0[-3000:]
    a, b = st.load_file(ref_out), st.load_file(dp_out)
    for k in a:
        assert torch.allclose(a[k], b[k], atol=1e-2, rtol=1e-2), (extra, k, (a[k] - b[k]).abs().max())


def test_native_lora_bucket_launched_inside_backward():
    """LoRA on GPT-2-tiny, 2 loopback ranks: the single fused bucket's all-reduce is issued by the grad-ready hook
    of its last parameter -- before the backward ends -- not by the post-backward sweep."""
    lora = ["--random_init", "--model", "gpt2-tiny", "--synthetic_data", "--synthetic_tokens", "100000", "--seq_len",
            "64", "--lr", "1e-3", "--log_interval", "1", "--deterministic", "--steps", "3", "--batch_size", "4"]
    res = _run_ranks([_bin("gpt2_lora_finetune"), *lora], 2)
    for rc, o, e in res:
        assert rc == 0, o[-2000:] + e[-2000:]
    assert "[dp] first step: 1 of 1 bucket" in res[0][1], res[0][1][-3000:]
