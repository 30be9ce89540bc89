import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

# Hot-path parity runs first, so that under `pytest -x`
# a failure in a peripheral subsystem (C++ example, denoiser, gather) can never
# leave the path tracer's own oracle-parity tests unreached.
FIRST = ("test_gpu_parity.py", "test_ref_scenes.py", "test_gpu_fullsize.py", "test_formats_gpu.py",
         "test_emitters.py")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")
    config.addinivalue_line("markers", "slow: long-running")


def _has_gpu():
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:
        return False


def _rank(item):
    name = os.path.basename(str(item.fspath))
    return FIRST.index(name) if name in FIRST else len(FIRST)


def pytest_collection_modifyitems(config, items):
    items.sort(key=_rank)  # stable: file-internal order is kept
    if _has_gpu():
        return
    skip = pytest.mark.skip(reason="no HIP device")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)
