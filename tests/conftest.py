import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs a real MI355X (gfx950) and the built HIP extension')
    config.addinivalue_line('markers', 'slow: long-running test')


@pytest.fixture(scope='session')
def gpu_ops():
    """The compiled HIP extension; GPU tests must never silently fall back to eager torch."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    from dotaclient_amd import ops
    return ops.require()
