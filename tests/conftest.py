import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box via gpurun)")
    config.addinivalue_line("markers", "slow: multi-process or long-running test")
    # under pytest-xdist each worker gets its share of the CPUs: every worker running torch's
    # default thread pool (all CPUs) oversubscribes the box ~N-fold and the CPU training tests
    # crawl
    n = int(os.environ.get("PYTEST_XDIST_WORKER_COUNT", "0") or 0)
    if n > 1:
        import torch

        torch.set_num_threads(max(1, (os.cpu_count() or 1) // n))


def pytest_collection_modifyitems(config, items):
    import torch

    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this container")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)
