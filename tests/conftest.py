import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "karpenter-provider-aws_amd"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")


@pytest.fixture(scope="session")
def lib():
    import kpamd
    return kpamd.load_lib()


@pytest.fixture(scope="session")
def catalog(lib):
    from kpamd import catalog as c
    return c.build_catalog(lib)


@pytest.fixture(scope="session")
def ctx():
    import kpamd
    c = kpamd.Context(0)
    yield c
    c.close()


@pytest.fixture(params=["batch", "single"])
def general_mode(request, monkeypatch):
    """The general consolidation path two ways: the superset Solve with batched simulations (default), and every
    subset compiled on its own (KP_GENERAL_BATCH=0)."""
    monkeypatch.setenv("KP_GENERAL_BATCH", "1" if request.param == "batch" else "0")
    return request.param
