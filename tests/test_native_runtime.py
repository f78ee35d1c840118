"""Native host-runtime self-test (csrc/tests/runtime_selftest.cpp) built plain and under
AddressSanitizer + UndefinedBehaviorSanitizer.  Covers the C++ JSON parser,
safetensors writer/reader incl. 200 corrupted-header variants, byte-level / SentencePiece BPE
round trips, the token dataset (DP sharding, resume) and the PowerMonitor policy."""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host C++ compiler")
def test_runtime_selftest_asan_ubsan(tmp_path):
    r = subprocess.run(["bash", os.path.join(REPO, "scripts", "sanitize_runtime.sh"), str(tmp_path)],
                       capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    assert "sanitized runtime selftest OK" in r.stdout
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error:" not in r.stderr


def test_energy_module_policy():
    """`mobilefinetuner_amd.energy` facade over the native PowerMonitor (reference power_monitor.cpp:70-112)."""
    from mobilefinetuner_amd import energy
    c = energy.PowerConfig()
    c.check_interval_steps = 1
    m = energy.PowerMonitor(c)
    m.set_manual_readings(100, 30)
    cool = m.suggest_sleep_ms(1)
    m.set_manual_readings(10, 50)  # low battery + hot -> slower target frequency -> longer sleep
    assert m.suggest_sleep_ms(2) > cool


def test_mfu_counters():
    from mobilefinetuner_amd.models.gpt2 import GPT2Config
    from mobilefinetuner_amd.utils import trace
    fpt = trace.model_flops_per_token_cfg(GPT2Config.preset("gpt2"), 128, 124_439_808, 442_368)
    # 4N + 2N_trainable + attention (12 layers x 2 x 128 x 768 x 3)
    assert abs(fpt - (4 * 124_439_808 + 2 * 442_368 + 12 * 2 * 128 * 768 * 3)) < 1
    tf, frac = trace.mfu(1e6, fpt)
    assert abs(tf - fpt * 1e6 / 1e12) < 1e-9 and abs(frac - tf / 2500.0) < 1e-12


def test_lora_dy_grids_fit_one_round():
    """lora_dy / lora_xty grids (2 resident 68-KB workgroups per CU on 256 CUs) never exceed one round:
    round 3 sized GPT-2's 768 / 2304 and Gemma-3's 640-wide operands to 513 workgroups, the last of which
    ran alone after the first round.  Host-side sizing only (no GPU needed)."""
    from mobilefinetuner_amd._ext import native
    C = native()
    for M, N in [(131072, 2304), (131072, 768), (65536, 640), (65536, 1024), (65536, 2048), (65536, 256),
                 (512, 2304), (7, 768)]:
        blocks = C.lora_dy_grid_blocks(M, N)
        assert 1 <= blocks <= 512, (M, N, blocks)
        if M >= 65536:
            assert blocks >= 384, (M, N, blocks)  # still fills most of the 512 slots
