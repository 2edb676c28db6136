import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (HIP) device')


@pytest.fixture(scope='session')
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.fail('gpu test selected but no HIP device is visible')
    return torch.device('cuda:0')


@pytest.fixture
def knob():
    """set(name, value): a libsr_hip tuning knob (sr_set_knob) for this test, restored at teardown."""
    from basicsr4rs_amd import _lib
    held = []

    def set_(name, value):
        k = _lib.knob(name, value)
        k.__enter__()
        held.append(k)

    yield set_
    for k in reversed(held):
        k.__exit__(None, None, None)
