import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through the HIP C-ABI library)")
    config.addinivalue_line("markers", "slow: long CPU test")


def gpu_available() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def kat():
    import json
    with open(os.path.join(ROOT, "tests", "golden", "kat_reference.json")) as f:
        return json.load(f)


@pytest.hookimpl(trylast=True)  # after -m deselection
def pytest_collection_modifyitems(session, config, items):
    """GPU sessions: bring up torch's HIP runtime before the first test touches libhipbls.

    torch ships its own libamdhip64/libhsa-runtime64 (no SONAME shared with /opt/rocm's, which libhipbls links), so a
    process that uses both holds two HIP runtimes.  bench.py always initializes torch's first; a test session whose
    first GPU user is libhipbls could leave torch's later device enumeration failing ("No HIP GPUs are available",
    seen once after the RLC tests ran first).  Initializing torch up front gives every GPU session bench.py's order."""
    if not any(item.get_closest_marker("gpu") for item in items):
        return
    # the library the GPU tests load must be built from the sources beside it: the box runs the
    # pushed binary, so a stale one would test other code than HEAD's
    from charon_amd import build
    try:
        build.verify()
    except RuntimeError as e:
        raise pytest.UsageError(str(e))
    try:
        import torch
        if torch.cuda.is_available():
            torch.zeros(1, device="cuda")
    except Exception:
        pass
