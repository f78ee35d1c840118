import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
# the fp32 host oracle (tests/oracle) serves host-tensor calls of the op layer in this process and,
# through the environment, in every subprocess a test starts (gloo ranks, bench --cpu_smoke)
os.environ.setdefault("MFT_HOST_ORACLE", os.path.join(os.path.dirname(os.path.abspath(__file__)), "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: long-running test")


def pytest_collection_modifyitems(config, items):
    import torch
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this environment")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)
