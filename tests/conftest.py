import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")
for p in (REPO, os.path.join(REPO, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 GPU (MI355X)")
    config.addinivalue_line("markers", "slow: long-running")


def pytest_runtest_logstart(nodeid, location):
    """On a gpurun box ($GRAFT_REPO_ROOT), the test being started is appended to
    gpurun_out/progress.log: a long multi-rank test shows progress there, and a hung one is named."""
    root = os.environ.get("GRAFT_REPO_ROOT")
    if root:
        import time

        os.makedirs(os.path.join(root, "gpurun_out"), exist_ok=True)
        with open(os.path.join(root, "gpurun_out", "progress.log"), "a") as fh:
            fh.write(f"{time.strftime('%H:%M:%S')} {nodeid}\n")


def progress(msg: str) -> None:
    """A line in gpurun_out/progress.log from inside a long test (no-op off the box)."""
    root = os.environ.get("GRAFT_REPO_ROOT")
    if root:
        import time

        with open(os.path.join(root, "gpurun_out", "progress.log"), "a") as fh:
            fh.write(f"{time.strftime('%H:%M:%S')}   {msg}\n")


@pytest.fixture(scope="session")
def golden():
    return GOLDEN


@pytest.fixture(scope="session")
def manifest():
    import json

    with open(os.path.join(GOLDEN, "manifest.json")) as fh:
        return json.load(fh)
