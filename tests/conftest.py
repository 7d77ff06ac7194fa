import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

# the reference's bundled 10k-record validation file (data/val.tfrecords), shipped with the tests
# so that the GPU box (no /root/reference there) runs the data-driven tests too
REF_DATA = os.path.join(os.path.dirname(os.path.abspath(__file__)), "fixtures", "val.tfrecords")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run via gpurun)")
    config.addinivalue_line("markers", "slow: long-running test")


def gpu_available() -> bool:
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:  # pragma: no cover
        return False


@pytest.fixture(scope="session")
def ref_data_path():
    if not os.path.exists(REF_DATA):
        pytest.skip("tests/fixtures/val.tfrecords not available")
    return REF_DATA
