import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; runs the HIP path through the C ABI")
    config.addinivalue_line("markers", "slow: longer CPU tests")


@pytest.fixture(scope="session")
def hip_ctx():
    """One HIP context for the whole GPU session (tests run in one process on the GPU box)."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from srsran_projectvtlmo_amd import _lib
    ctx = _lib.Context(0, max_queue_cbs=256, nof_harq_slots=0)
    yield ctx
    ctx.close()


@pytest.fixture(scope="session")
def hip_ctx_harq():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from srsran_projectvtlmo_amd import _lib
    ctx = _lib.Context(0, max_queue_cbs=256, nof_harq_slots=512)
    yield ctx
    ctx.close()
