"""The test-suite's fp32 PyTorch oracle (host tensors only, never shipped on the GPU path).

* ``reference`` -- plain-PyTorch fp32 reference math of every fused op: the numerics oracle the
  HIP kernels are compared against (tests/test_kernels_gpu.py, tests/test_models_gpu.py).
* ``host_ops`` -- the public op layer's signatures implemented on that math, installed into
  ``mobilefinetuner_amd.ops.functional`` (``install()``, or ``MFT_HOST_ORACLE=<this dir>`` for
  subprocesses) so the GPU-less CI can run whole models on the CPU: HF-parity tests, gloo data
  parallelism, CLI smoke runs.  The package's op layer itself has a single (GPU) device path.
"""
from . import host_ops, reference  # noqa: F401

ORACLE_DIR = __path__[0]


def install():
    from mobilefinetuner_amd.ops import functional as Fx
    Fx.install_host_ops(host_ops)
