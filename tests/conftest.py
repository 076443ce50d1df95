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


@pytest.fixture
def ov(ctx):
    """kp_ctx_set_overrides on the session context for one test (keyword fields of kp_overrides); every override is
    reset to the production choice after the test."""
    yield ctx.set_overrides
    ctx.set_overrides()


@pytest.fixture(params=["batch", "single"])
def general_mode(request, ov):
    """The general consolidation path two ways: the superset Solve with batched simulations (default), and every
    subset compiled on its own (kp_overrides.general_batch = 1)."""
    ov(general_batch=0 if request.param == "batch" else 1)
    return request.param
