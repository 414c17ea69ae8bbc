import os
import sys

import pytest
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an AMD GPU (MI355X) and the HIP extension')
    config.addinivalue_line('markers', 'multigpu: needs at least 2 GPUs')


@pytest.fixture(autouse=True)
def manual_seed_zero():
    torch.manual_seed(0)


@pytest.fixture(scope='session')
def gpu_sleep():
    """Spin the current GPU stream for `seconds` (HIP spin kernel, K5)."""
    from torchgpipe_amd.ops import misc

    def sleep(seconds, device=None):
        misc.spin(seconds, device or torch.device('cuda', torch.cuda.current_device()))
    return sleep


def pytest_report_header():
    return f'torch: {torch.__version__} hip: {torch.version.hip}'
