import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, 'tests', 'golden')):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (HIP extension, cuda:0)')


import gc  # noqa: E402

import pytest  # noqa: E402


@pytest.fixture(autouse=True)
def _release_device_memory():
    """After every test: drop the test's tensors and hand the caching allocator's blocks back to
    the device. The real-size C3 / C5 tests leave ~100 GB cached in this process otherwise, which
    the multi-process tests' spawned ranks (their own allocators, the same GPU) then cannot get."""
    yield
    import torch
    if torch.cuda.is_initialized():
        gc.collect()
        torch.cuda.empty_cache()
