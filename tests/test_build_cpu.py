"""Build hygiene (CPU): the torch-free part of the framework -- the kernels, the libmft engine and the native
CLIs -- builds and imports without torch; only the PyTorch-driven oracle package's _C.so needs it."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_package_import_and_native_build_driver_do_not_import_torch():
    code = ("import sys; import mobilefinetuner_amd, mobilefinetuner_amd._build as b; "
            "assert 'torch' not in sys.modules, 'torch imported'; "
            "assert callable(b.build_native); print('ok')")
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "ok" in r.stdout, r.stdout + r.stderr


def test_native_build_links_no_vendor_gemm_library():
    """The native CLIs run every GEMM on the hand-written kernels: no hipBLASLt / rocBLAS in their link."""
    exe = os.path.join(ROOT, "mobilefinetuner_amd", "bin", "gpt2_lora_finetune")
    if not os.path.exists(exe):
        import pytest
        pytest.skip("native CLIs not built")
    r = subprocess.run(["ldd", exe], capture_output=True, text=True, timeout=60)
    libs = r.stdout
    assert "hipblaslt" not in libs.lower() and "rocblas" not in libs.lower(), libs
