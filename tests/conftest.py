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


def torch_runtime_mapped():
    """paths of torch's bundled HIP runtime / RCCL mapped into this process
    (the product library links /opt/rocm's; the GPU parity tests must run on
    the runtime the bench uses)"""
    try:
        maps = open("/proc/self/maps").read().split("\n")
    except OSError:
        return []
    return sorted({ln.split()[-1] for ln in maps
                   if "/torch/" in ln and ("libamdhip64" in ln or "librccl" in ln) and "/" in ln})


def runtime_mapped():
    """the HIP runtime and RCCL libraries this process has mapped"""
    try:
        maps = open("/proc/self/maps").read().split("\n")
    except OSError:
        return []
    return sorted({ln.split()[-1] for ln in maps if ("libamdhip64" in ln or "librccl" in ln) and "/" in ln})


@pytest.fixture(scope="session")
def hip():
    """The C-ABI library, initialised on device 0 (GPU tests only).  Fails the
    session if torch's own HIP runtime or RCCL is mapped into the pytest
    process, before or after the GPU tests (only /opt/rocm's may be)."""
    bad = torch_runtime_mapped()
    if bad:
        pytest.fail(f"torch's HIP runtime / RCCL mapped into the GPU test process: {bad}")
    import pagedattn
    pagedattn.init(int(os.environ.get("HPA_DEVICE", "0")))
    print(f"[conftest] GPU tests on {runtime_mapped()}")
    yield pagedattn
    bad = torch_runtime_mapped()
    if bad:
        pytest.fail(f"torch's HIP runtime / RCCL mapped into the GPU test process: {bad}")
