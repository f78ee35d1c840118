"""GPU-less CI of the native engine's multi-rank bookkeeping, built with the CMake
"tsan" preset (host C++ instrumented with ThreadSanitizer; HIP kernels compiled but never launched):
csrc/tests/engine_host_selftest.cpp runs plan_flat's bucket / chunk / replicated-fp32 layout at world
1..8, the ZeRO-3 unit partitions (plan_zero3), and the loopback communicator in host-only mode with
4 ranks as threads -- TCP star bootstrap, every collective (all-reduce sum / max / avg in fp32, bf16,
int32; reduce-scatter; all-gather in place; broadcast; 200 back-to-back tags), the watchdog's idle
timer (setup not timed, quiet scopes) -- plus the allocator and autograd tape checks.  Any data race
in the comm / watchdog threads fails the run (halt_on_error)."""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("cmake") is None or shutil.which("ninja") is None, reason="cmake / ninja missing")
def test_engine_host_selftest_under_tsan():
    bdir = os.path.join(REPO, "build", "cmake-tsan")
    r = subprocess.run(["cmake", "--preset", "tsan"], cwd=REPO, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    r = subprocess.run(["cmake", "--build", "--preset", "tsan", "--target", "engine_host_selftest"], cwd=REPO,
                       capture_output=True, text=True, timeout=1800)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 second_deadlock_stack=1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([os.path.join(bdir, "engine_host_selftest")], cwd=bdir, capture_output=True, text=True,
                       timeout=600, env=env)
    out = r.stdout + r.stderr
    assert r.returncode == 0 and "engine_host_selftest: PASS" in r.stdout, out[-4000:]
    assert "WARNING: ThreadSanitizer" not in out, out[-4000:]
    assert "[comm] host-only loopback: 4 ranks" in r.stdout
