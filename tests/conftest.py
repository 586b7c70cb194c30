import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C ABI)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def golden():
    import json

    with open(os.path.join(ROOT, "tests", "golden", "ref_vectors.json")) as f:
        return json.load(f)


@pytest.fixture(autouse=True)
def _gpu_results_came_from_the_gpu(request):
    """Every -m gpu test: the scalar hooks' CPU fallback (used only when the
    GPU path fails) must not have answered anything during the test."""
    if request.node.get_closest_marker("gpu") is None:
        yield
        return
    import torch

    if not torch.cuda.is_available():
        yield
        return
    import val_protocol_amd.crc as vc

    before = vc.cpu_fallback_count()
    yield
    assert vc.cpu_fallback_count() == before, "a scalar hook fell back to the CPU during a GPU test"
