"""Device parity at BASELINE.json's full sizes, against oracle results committed as fixtures
(tests/golden/fullsize_digests.json, generated in this container by tests/golden/make_fullsize_digests.py from the
same generators and seeds): the headline config 2 at 50k pods, config 3 at 100k pods onto 5k existing nodes, and
config 5 at 100k pods (17.5k NodeClaims: the newNodeClaims order spills past the device's LDS capacity by itself),
config 5 at 100k pods with its pools' cpu limits divided by 10 (the regime where the 1M-pod burst ends: NodePool limits
bind, 38.9 % of the pods unschedulable), config 5 at 1M pods when its digest has been generated, config 4's 10k-node cluster on every firstNConsolidationOption prefix plus 200 random candidate subsets.

The -m "not gpu" test checks the fixture is consistent with the generators (counts and shapes)."""
import json
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))


@pytest.fixture(scope="module")
def digests():
    return json.load(open(os.path.join(HERE, "golden", "fullsize_digests.json")))


def test_fixture_shape(digests):
    assert digests["config2-50000"]["placed"] == 50_000
    assert digests["config3-100000"]["on_existing"] > 0
    assert digests["config5-100000"]["nodeclaims"] > 2 * 8192, "past the device's LDS sort capacity without forcing it"
    lim = digests["config5-limits-100000"]
    assert 100_000 - lim["placed"] >= 25_000, "NodePool limits bind: at least 25 % of the pods end unschedulable"
    if "config5-1000000" in digests:
        assert 1_000_000 - digests["config5-1000000"]["placed"] >= 250_000
    c4 = digests["config4-10000"]
    assert len(c4["prefixes"]) == 100 and len(c4["random"]) == 200
    decisions = {r[0] for r in c4["random"]}
    assert decisions >= {1, 2}, "the near-capacity cluster yields deletes and replacements"


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["config2-50000", "config2-burst-50000", "config3-100000", "config5-100000",
                                  "config5-limits-100000", "config5-1000000"])
def test_solve_fullsize(ctx, catalog, digests, name):
    import kpamd
    import make_fullsize_digests as mk
    if name not in digests:
        pytest.skip(f"{name}: digest not generated (make_fullsize_digests.py {name})")
    prob = mk._solves()[name](catalog)
    res = kpamd.Scheduler(ctx, prob).solve()
    got = mk.solve_digest(res)
    assert got == digests[name]
    if name in ("config5-100000", "config5-1000000"):
        assert len(res["nodeclaims"]) > 8192
        assert res["stats"]["order_chunks"][4] == 2, "the chunked order past the LDS capacity"


@pytest.mark.gpu
def test_consolidation_fullsize(ctx, catalog, digests):
    import kpamd
    import make_fullsize_digests as mk
    from kpamd import synth
    cl = synth.config4(catalog, n_nodes=10_000, seed=4)
    pre, rnd = mk.config4_subsets(cl)
    plan = kpamd.ClusterPlan(ctx, cl)
    try:
        res, _ = plan.simulate(pre + rnd)
    finally:
        plan.close()
    want = digests["config4-10000"]
    got = [mk.sim_record(r) for r in res]
    assert got[:len(pre)] == want["prefixes"]
    assert got[len(pre):] == want["random"]


@pytest.mark.gpu
def test_general_fullsize(ctx, catalog, digests):
    """The general path at the bench's size: 2,000-node spread cluster, 300 subsets batched on the superset Solve,
    every decision field equal to the oracle's digest."""
    import kpamd
    import make_fullsize_digests as mk
    from kpamd import synth
    if "general-2000" not in digests:
        pytest.skip("general-2000: digest not generated (make_fullsize_digests.py general-2000)")
    cl = synth.spread_cluster(catalog, 2_000)
    pre, rnd = mk.general_subsets(cl)
    plan = kpamd.ClusterPlan(ctx, cl)
    try:
        res, st = plan.simulate(pre + rnd)
    finally:
        plan.close()
    assert st["phase_cycles"][:2] == [len(pre) + len(rnd), 0], "every subset batched"
    want = digests["general-2000"]
    got = [mk.sim_record(r) for r in res]
    assert got[:len(pre)] == want["prefixes"]
    assert got[len(pre):] == want["random"]


@pytest.mark.gpu
def test_general_10000(ctx, catalog, digests):
    """The general path at config 4's size: the 10,000-node spread cluster (83k pods), the 100 prefixes and 200 random
    subsets of 2..100 candidates, batched on the superset Solve, every decision field equal to the oracle's digest."""
    import kpamd
    import make_fullsize_digests as mk
    from kpamd import synth
    if "general-10000" not in digests:
        pytest.skip("general-10000: digest not generated (make_fullsize_digests.py general-10000)")
    cl = synth.spread_cluster(catalog, 10_000)
    pre, rnd = mk.general10k_subsets(cl)
    plan = kpamd.ClusterPlan(ctx, cl)
    try:
        res, st = plan.simulate(pre + rnd)
    finally:
        plan.close()
    assert st["phase_cycles"][:2] == [len(pre) + len(rnd), 0], "every subset batched"
    want = digests["general-10000"]
    got = [mk.sim_record(r) for r in res]
    assert got[:len(pre)] == want["prefixes"]
    assert got[len(pre):] == want["random"]
