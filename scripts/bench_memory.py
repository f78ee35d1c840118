#!/usr/bin/env python3
"""Memory / energy A/B benchmarks (the reference's scripts/benchmark/test_all_models_sharding.sh,
test_sharding_aggressive.sh and test_energy_function.sh, SURVEY §6 'benchmark methodology').

  sharding : each model trained for a few LoRA steps (batch 2, seq 128, rank 8, alpha 16, lr 1e-4:
             the reference's settings) without and with ``--shard_enable --shard_budget_mb B``;
             reports peak device memory (torch max_memory_allocated, from the CLI's metrics JSONL),
             peak host RSS of the child (getrusage ru_maxrss) and wall time -- the reference's table
             measured peak process RSS of a CPU run (README.md:404-411); on MI355X the weights live in
             HBM, so the device peak is the quantity the sharder bounds, and the pinned host tier shows
             up in the host RSS.
  energy   : 10 steps with and without ``--pm_schedule 0-:200`` (200 ms sleep per step): the added
             wall time must be about 10 x 200 ms (test_energy_function.sh:160-168).

  python scripts/bench_memory.py sharding [--models gpt2,gpt2-medium,gemma3-270m,gemma3-1b] [--budget_mb 300]
  python scripts/bench_memory.py energy
Writes one JSON line per run to stdout (and --out FILE).
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_cli(args, metrics):
    env = dict(os.environ)
    env["PYTHONPATH"] = REPO + os.pathsep + env.get("PYTHONPATH", "")
    log = metrics + ".log"
    t0 = time.perf_counter()
    with open(log, "w") as lf:
        p = subprocess.Popen([sys.executable, "-m", *args, "--metrics_out", metrics], cwd=REPO, env=env,
                             stdout=lf, stderr=subprocess.STDOUT)
        _, status, ru = os.wait4(p.pid, 0)  # this child's own rusage (peak RSS)
    wall = time.perf_counter() - t0
    if os.waitstatus_to_exitcode(status) != 0:
        raise RuntimeError(f"{' '.join(args)} failed:\n{open(log).read()[-4000:]}")
    recs = [json.loads(x) for x in open(metrics)] if os.path.exists(metrics) else []
    hbm = max((x.get("hbm_peak_gb", 0.0) for x in recs), default=0.0)
    # steady-state throughput (setup -- model build, host-tier registration -- excluded): median
    # tokens/s of the logged steps after the first three
    tps = sorted(x["tokens_per_sec"] for x in recs[3:] if x.get("tokens_per_sec"))
    med = tps[len(tps) // 2] if tps else 0.0
    return {"wall_s": round(wall, 2), "hbm_peak_gb": round(hbm, 3), "host_rss_peak_gb": round(ru.ru_maxrss / 2 ** 20, 3),
            "steps_logged": len(recs), "steady_tokens_per_s": round(med, 1)}


def cli_for(model):
    if model.startswith("gemma"):
        return ["mobilefinetuner_amd.cli.train_lora_gemma", "--model", model, "--batch", "2", "--seq_len", "128",
                "--lr", "1e-4", "--rank", "8", "--alpha", "16", "--targets", "full"]
    return ["mobilefinetuner_amd.cli.gpt2_lora_finetune", "--model", model, "--batch_size", "2", "--seq_len", "128",
            "--lr", "1e-4", "--rank", "8", "--alpha", "16"]


def steps_flag(model, n):
    return ["--max_steps", str(n)] if model.startswith("gemma") else ["--steps", str(n)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=["sharding", "energy"])
    ap.add_argument("--models", default="gpt2,gpt2-medium,gemma3-270m,gemma3-1b")
    ap.add_argument("--budget_mb", type=int, default=300)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    common = ["--random_init", "--synthetic_data", "--synthetic_tokens", "200000", "--log_interval", "1", "--no_graph"]
    rows = []
    with tempfile.TemporaryDirectory() as td:
        if a.mode == "sharding":
            for m in [x for x in a.models.split(",") if x]:
                for shard in (False, True):
                    extra = ["--shard_enable", "--shard_budget_mb", str(a.budget_mb)] if shard else []
                    met = os.path.join(td, f"{m}_{int(shard)}.jsonl")
                    res = run_cli(cli_for(m) + steps_flag(m, a.steps) + common + extra, met)
                    rows.append({"bench": "sharding", "model": m, "shard": shard,
                                 "budget_mb": a.budget_mb if shard else None, **res})
                    print(json.dumps(rows[-1]), flush=True)
        else:
            m = a.models.split(",")[0]
            for sched in ("", "0-:200"):
                extra = ["--pm_schedule", sched] if sched else []
                met = os.path.join(td, f"energy_{bool(sched)}.jsonl")
                res = run_cli(cli_for(m) + steps_flag(m, 10) + common + extra, met)
                rows.append({"bench": "energy", "model": m, "pm_schedule": sched or None, **res})
                print(json.dumps(rows[-1]), flush=True)
            added = rows[1]["wall_s"] - rows[0]["wall_s"]
            print(json.dumps({"bench": "energy", "added_wall_s": round(added, 2), "expected_s": 2.0}), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            for r in rows:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
