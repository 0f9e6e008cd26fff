import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN_DIR = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def golden():
    with open(os.path.join(GOLDEN_DIR, "golden.json")) as f:
        meta = json.load(f)
    arrays = dict(np.load(os.path.join(GOLDEN_DIR, "golden.npz")))
    return meta, arrays


@pytest.fixture(autouse=True)
def _one_blas_thread(request):
    """CPU tests run the oracle with one BLAS thread: its small QR / GEMV calls gain nothing from
    threads (and contend with other jobs), and the golden fixtures were generated that way
    (tests/golden/make_golden.py, OPENBLAS_NUM_THREADS=1).  Tests that vary the thread count set their
    own limits inside; GPU tests keep the machine's default."""
    if request.node.get_closest_marker("gpu"):
        yield
        return
    from threadpoolctl import threadpool_limits
    with threadpool_limits(limits=int(os.environ.get("GNK_TEST_BLAS_THREADS", "1")), user_api="blas"):
        yield
