"""Launch-side selection oracle (instance.DefaultProvider.Create, R:pkg/providers/instance/instance.go:117-125):
filterInstanceTypes (:242-270) -> getCapacityType (:504-518) -> getOverrides (:392-439), pinned to the behaviour
the reference's own launch tests assert (R:pkg/providers/instancetype/suite_test.go:409-597) on a one-pod Solve
over the docs catalogue, and to the per-filter kept sets of R:pkg/providers/instance/filter/filter_test.go
(tests/test_filters_golden.py) through the shared filter code."""
import numpy as np
import pytest

K = "karpenter.k8s.aws/"
ONE_CPU = {"cpu": 1000, "pods": 1000}


@pytest.fixture(scope="module")
def cat():
    import kpamd
    from kpamd import catalog
    return catalog.build_catalog(kpamd.load_lib())


def launch_one_pod(cat, pool_reqs, requests=ONE_CPU):
    """Solve one pod (ExpectProvisioned), then Create's launch selection for its NodeClaim."""
    import kpamd
    from kpamd import catalog, synth
    from oracle import pyoracle
    prob = synth.single_pod_problem(cat, pool_reqs, requests)
    res = pyoracle.solve(prob)
    assert len(res["nodeclaims"]) == 1
    out = pyoracle.launch_select(cat, kpamd.launch_requests_from_solve(res), catalog.ZONES)
    return prob, res, out[0]


def order_by_price(cat, reqs_types, price_of):
    return sorted(reqs_types, key=lambda t: (price_of(t), cat[t].name))


def test_cheapest_100_then_60(cat):
    """suite_test.go:409-453: overrides come from the 100 cheapest types (OrderByPrice over the pool
    requirements, name tie-break) and launch exactly maxInstanceTypes = 60 of them."""
    pool = [("karpenter.sh/capacity-type", "In", ["on-demand"])]
    _, res, out = launch_one_pod(cat, pool)
    assert out["status"] == 0 and out["capacity_type"] == "on-demand"
    assert len(out["types"]) == 60
    cheapest100 = set(res["nodeclaims"][0]["options"][:100])
    assert set(out["types"]) <= cheapest100
    assert {t for t, _ in out["overrides"]} == set(out["types"])


def test_spot_cheaper_than_cheapest_od(cat):
    """suite_test.go:454-525: capacity type In {spot, on-demand} launches spot, and the spot types kept are
    those with a spot offering no dearer than the cheapest compatible on-demand offering (SpotInstanceFilter,
    R:filter.go:372-380). The reference test's fake pricing is uniform per type, so it can assert this per
    override; with per-zone spot prices the guarantee is per type (its cheapest spot offering)."""
    pool = [("karpenter.sh/capacity-type", "In", ["spot", "on-demand"])]
    _, _, out = launch_one_pod(cat, pool)
    assert out["status"] == 0 and out["capacity_type"] == "spot" and out["rejected_spot"] > 0
    od = min(o.price for t in out["types"] for o in cat[t].offerings if o.capacity_type == "on-demand")
    for t in out["types"]:
        assert min(o.price for o in cat[t].offerings if o.capacity_type == "spot") <= od
    assert {z for _, z in out["overrides"]} <= set(["test-zone-1a", "test-zone-1b", "test-zone-1c"])


def test_minvalues_keeps_metal(cat):
    """suite_test.go:531-560: a requirement with minValues disables the exotic filter, so metal types launch."""
    pool = [("karpenter.sh/capacity-type", "In", ["spot"], 1), (K + "instance-category", "In", ["c", "m", "r"])]
    _, _, out = launch_one_pod(cat, pool, {"cpu": 60000, "pods": 1000})
    assert out["status"] == 0 and out["rejected_exotic"] == 0
    assert any("metal" in cat[t].name for t in out["types"])


def test_deprioritize_metal_and_gpu(cat):
    """suite_test.go:561-597: without minValues the exotic filter drops metal and GPU types."""
    pool = [("karpenter.sh/capacity-type", "In", ["on-demand"])]
    _, res, out = launch_one_pod(cat, pool, {"cpu": 60000, "pods": 1000})
    assert out["status"] == 0
    opts = res["nodeclaims"][0]["options"]
    assert any("metal" in cat[t].name for t in opts), "scenario must offer metal types"
    assert out["rejected_exotic"] > 0
    for t in out["types"]:
        assert "metal" not in cat[t].name
        assert not cat[t].name.startswith(("g", "p"))


def test_gpu_request_launches_gpu(cat):
    """All remaining types are exotic (GPU request): the exotic filter keeps them (R:filter.go:309-312)."""
    pool = [("karpenter.sh/capacity-type", "In", ["on-demand"])]
    _, _, out = launch_one_pod(cat, pool, {"cpu": 1000, "pods": 1000, "nvidia.com/gpu": 1000})
    assert out["status"] == 0 and out["rejected_exotic"] == 0 and len(out["types"]) > 0


def test_insufficient_capacity(cat):
    """CompatibleAvailableFilter leaving nothing -> InsufficientCapacityError (R:instance.go:255-257)."""
    from kpamd import catalog
    from oracle import pyoracle
    req = ([("karpenter.sh/capacity-type", "In", ["on-demand"])], {"cpu": 10 ** 9}, list(range(len(cat))))
    out = pyoracle.launch_select(cat, [req], catalog.ZONES)[0]
    assert out["status"] == 1 and out["failed_filter"] == 0
    out = pyoracle.launch_select(cat, [(req[0], {"cpu": 1000}, [])], catalog.ZONES)[0]
    assert out["status"] == 1 and out["failed_filter"] == 0


def test_subnet_zones_restrict_overrides(cat):
    """getOverrides keeps only offerings whose zone has a subnet (zonalSubnets, R:instance.go:423-426)."""
    import kpamd
    from kpamd import catalog
    from oracle import pyoracle
    pool = [("karpenter.sh/capacity-type", "In", ["on-demand"])]
    _, res, _ = launch_one_pod(cat, pool)
    rq = kpamd.launch_requests_from_solve(res)
    one = pyoracle.launch_select(cat, rq, catalog.ZONES[:1])[0]
    assert one["overrides"] and all(z == catalog.ZONES[0] for _, z in one["overrides"])
    none = pyoracle.launch_select(cat, rq, [])[0]
    assert none["status"] == 0 and none["overrides"] == []


def test_random_requests_invariants(cat):
    """Size-independent properties on random requests: types ⊆ request list, ≤ 60, ordered by price then name;
    overrides follow the type order; OD fallback warning only for on-demand launches flexible to spot."""
    from kpamd import catalog, synth
    from oracle import pyoracle
    reqs = synth.random_launch_requests(cat, 200, seed=3)
    outs = pyoracle.launch_select(cat, reqs, catalog.ZONES)
    statuses = set()
    for (r, _, lst), o in zip(reqs, outs):
        statuses.add(o["status"])
        if o["status"] != 0:
            assert o["types"] == []
            continue
        assert set(o["types"]) <= set(lst) and 0 < len(o["types"]) <= 60
        order = {t: i for i, t in enumerate(o["types"])}
        idx = [order[t] for t, _ in o["overrides"]]
        assert idx == sorted(idx)
        if o["od_fallback_warning"]:
            assert o["capacity_type"] == "on-demand" and len(o["types"]) < 5
    assert statuses >= {0, 1}
