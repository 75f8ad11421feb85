import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
os.environ.setdefault("MULTIGRAD_PROGRESS", "0")
# the engine tests were written against the full setup autotune (every candidate timed,
# however short the run); the library default budgets it to 10 % of the run, which
# tests/test_engine_cache_gpu.py covers explicitly
os.environ.setdefault("MULTIGRAD_AUTOTUNE", "on")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device + built _C extension)")
    config.addinivalue_line("markers", "slow: long-running test")


def pytest_collection_modifyitems(config, items):
    import torch
    have_gpu = torch.cuda.is_available()
    skip_gpu = pytest.mark.skip(reason="no HIP device")
    for item in items:
        if "gpu" in item.keywords and not have_gpu:
            item.add_marker(skip_gpu)
