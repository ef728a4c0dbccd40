import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "oracle"), os.path.join(REPO, "llm.c-paged_amd"),
          os.path.join(REPO, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")


@pytest.fixture(scope="session")
def hip():
    """The C-ABI library, initialised on device 0 (GPU tests only)."""
    import pagedattn
    pagedattn.init(int(os.environ.get("HPA_DEVICE", "0")))
    return pagedattn
