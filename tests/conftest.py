import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

# The scalar hooks answer inputs below the provider threshold on the CPU by
# design. The suite sets the threshold to 0 before the library loads, so
# every hook call a GPU test checks runs on the GPU (child processes inherit
# it); tests of the CPU engine set it explicitly (val_gpu_set_provider_min_bytes).
os.environ["VAL_GPU_PROVIDER_MIN_BYTES"] = "0"
# Likewise host-memory batch calls below the host-batch crossover run on the
# CPU engine by design; the GPU suite sends every one to the GPU.
os.environ["VAL_GPU_HOST_BATCH_MIN_BYTES"] = "0"


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

    before = vc.cpu_fallback_count(), vc.cpu_small_count(), vc.cpu_batch_count()
    yield
    vc.set_ragged_min_frames(-1)  # tests pin the binned path with vc.set_ragged_min_frames(1)
    assert vc.cpu_fallback_count() == before[0], "a scalar hook fell back to the CPU during a GPU test"
    assert vc.cpu_small_count() == before[1], "a scalar hook answered below the threshold during a GPU test"
    assert vc.cpu_batch_count() == before[2], "a host batch was answered by the CPU engine during a GPU test"
