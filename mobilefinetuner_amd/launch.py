"""mft_launch — single-node multi-process launcher with failure detection.

    python -m mobilefinetuner_amd.launch --nproc 8 [--master_port P] [--timeout S] script.py [args...]
    python -m mobilefinetuner_amd.launch --nproc 8 -m mobilefinetuner_amd.cli.gpt2_full_finetune [args...]

One process per GPU (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT in the
environment; the Python ranks build their RCCL communicator through torch.distributed's TCP store,
the native CLIs (bin/gpt2_lora_finetune, bin/gpt2_full_finetune) through libmft's own TCP unique-id
exchange, csrc/engine/comm.cpp).
SURVEY §5.3 "failure detection": the launcher watches every rank; when one exits non-zero (crash,
fault injection, RCCL watchdog abort) or the optional job timeout expires, the remaining ranks get
SIGTERM, then SIGKILL after a grace period, and the launcher exits with the failing rank's code, so a
dead rank never leaves its peers hanging inside a collective.  Each rank runs in its own process
group (killpg reaches its children too).  The reference has no multi-process runtime at all
(SURVEY §2.13).
"""
from __future__ import annotations

import argparse
import os
import signal
import socket
import subprocess
import sys
import time


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _terminate(procs, grace: float):
    for p in procs:
        if p.poll() is None:
            try:
                os.killpg(p.pid, signal.SIGTERM)
            except ProcessLookupError:
                pass
    t0 = time.time()
    while time.time() - t0 < grace and any(p.poll() is None for p in procs):
        time.sleep(0.05)
    for p in procs:
        if p.poll() is None:
            try:
                os.killpg(p.pid, signal.SIGKILL)
            except ProcessLookupError:
                pass
    for p in procs:
        try:
            p.wait(timeout=5)
        except subprocess.TimeoutExpired:
            pass


def launch(cmd, nproc: int, master_port: int = 0, timeout: float = 0.0, grace: float = 10.0,
           extra_env: dict | None = None) -> int:
    """Run ``cmd`` (argv list, without the python executable) on ``nproc`` ranks; returns the job's
    exit code (0 when every rank succeeded, else the first failing rank's code; 124 on timeout)."""
    port = master_port or _free_port()
    procs = []
    for r in range(nproc):
        env = dict(os.environ)
        env.update({"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(nproc), "LOCAL_WORLD_SIZE": str(nproc),
                    "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port),
                    # a rank stuck in a collective whose peer died raises instead of hanging
                    "TORCH_NCCL_ASYNC_ERROR_HANDLING": env.get("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")})
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        if extra_env:
            env.update(extra_env)
        procs.append(subprocess.Popen([sys.executable, *cmd], env=env, start_new_session=True))
    t0 = time.time()
    code = 0
    try:
        while True:
            states = [p.poll() for p in procs]
            failed = [(i, c) for i, c in enumerate(states) if c not in (None, 0)]
            if failed:
                i, code = failed[0]
                print(f"[mft_launch] rank {i} exited with code {code}; stopping the other ranks", file=sys.stderr,
                      flush=True)
                break
            if all(c == 0 for c in states):
                return 0
            if timeout > 0 and time.time() - t0 > timeout:
                print(f"[mft_launch] job exceeded {timeout:.0f}s; stopping all ranks", file=sys.stderr, flush=True)
                code = 124
                break
            time.sleep(0.1)
    except KeyboardInterrupt:
        code = 130
    _terminate(procs, grace)
    return code


def main(argv=None):
    ap = argparse.ArgumentParser(prog="mft_launch", description=__doc__.splitlines()[0])
    ap.add_argument("--nproc", "--nproc-per-node", type=int, default=1, dest="nproc")
    ap.add_argument("--master_port", "--master-port", type=int, default=0, dest="master_port")
    ap.add_argument("--timeout", type=float, default=0.0, help="whole-job wall-clock limit in seconds (0 = none)")
    ap.add_argument("--grace", type=float, default=10.0, help="seconds between SIGTERM and SIGKILL")
    ap.add_argument("-m", dest="module", default=None, help="run a module (like python -m)")
    ap.add_argument("script", nargs="?")
    ap.add_argument("args", nargs=argparse.REMAINDER)
    a = ap.parse_args(argv)
    if a.module:
        cmd = ["-m", a.module] + ([a.script] if a.script else []) + a.args
    elif a.script:
        cmd = [a.script] + a.args
    else:
        ap.error("give a script or -m module")
    return launch(cmd, a.nproc, a.master_port, a.timeout, a.grace)


if __name__ == "__main__":
    sys.exit(main())
