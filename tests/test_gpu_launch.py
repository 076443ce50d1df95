"""Launch-side selection on the device (kp_launch_select, launch_kernel) vs the oracle, bit-exact: status, failed
filter, counts per filter, capacity type, the launched types in order and the (type, zone) overrides in order."""
import pytest

pytestmark = pytest.mark.gpu


def run_both(ctx, cat, requests, zones, max_types=60):
    import kpamd
    from oracle import pyoracle
    ch = kpamd.Catalog(ctx, cat)
    plan = kpamd.LaunchPlan(ctx, ch, requests, zones, max_types=max_types)
    got, st = plan.run(read=True)
    plan.close()
    ch.close()
    want = pyoracle.launch_select(cat, requests, zones, max_types=max_types)
    return got, want, st


def check_same(got, want):
    assert len(got) == len(want)
    for i, (g, w) in enumerate(zip(got, want)):
        assert g == w, f"request {i}: device {g} vs oracle {w}"


@pytest.mark.parametrize("seed", range(4))
def test_random_requests(ctx, catalog, seed):
    from kpamd import catalog as cmod, synth
    reqs = synth.random_launch_requests(catalog, 300, seed=100 + seed)
    zones = [cmod.ZONES, cmod.ZONES[:2], cmod.ZONES[1:2], []][seed]
    got, want, st = run_both(ctx, catalog, reqs, zones)
    check_same(got, want)
    assert {g["status"] for g in got} >= {0, 1}
    assert st["attempts"] == sum(len(r[2]) for r in reqs)


@pytest.mark.parametrize("max_types", [1, 7, 100, 1024])
def test_max_types(ctx, catalog, max_types):
    from kpamd import catalog as cmod, synth
    reqs = synth.random_launch_requests(catalog, 120, seed=7)
    got, want, _ = run_both(ctx, catalog, reqs, cmod.ZONES, max_types=max_types)
    check_same(got, want)


@pytest.mark.parametrize("cfg", ["2", "5"])
def test_solve_nodeclaims(ctx, catalog, cfg):
    """The NodeClaims a Solve emits, launched: config 2 (selectors / affinity / tolerations) and config 5 (GPU and
    Neuron pools: exotic-only sets, minValues-free)."""
    import kpamd
    from kpamd import catalog as cmod, synth
    from oracle import pyoracle
    prob = synth.config2(catalog, n_pods=3000, seed=2) if cfg == "2" else synth.config5(catalog, n_pods=3000, seed=5)
    res = pyoracle.solve(prob)
    reqs = kpamd.launch_requests_from_solve(res)
    got, want, _ = run_both(ctx, catalog, reqs, cmod.ZONES)
    check_same(got, want)
    assert sum(g["capacity_type"] == "spot" for g in got) > 0


def test_reference_launch_kats_on_device(ctx, catalog):
    """The launch assertions of R:pkg/providers/instancetype/suite_test.go:409-597 through the device path."""
    import kpamd
    from kpamd import catalog as cmod, synth
    from oracle import pyoracle
    K = "karpenter.k8s.aws/"
    cases = [([("karpenter.sh/capacity-type", "In", ["on-demand"])], {"cpu": 1000, "pods": 1000}),
             ([("karpenter.sh/capacity-type", "In", ["spot", "on-demand"])], {"cpu": 1000, "pods": 1000}),
             ([("karpenter.sh/capacity-type", "In", ["spot"], 1), (K + "instance-category", "In", ["c", "m", "r"])],
              {"cpu": 60000, "pods": 1000}),
             ([("karpenter.sh/capacity-type", "In", ["on-demand"])], {"cpu": 60000, "pods": 1000})]
    reqs = []
    for pool, rq in cases:
        res = pyoracle.solve(synth.single_pod_problem(catalog, pool, rq))
        reqs += kpamd.launch_requests_from_solve(res)
    got, want, _ = run_both(ctx, catalog, reqs, cmod.ZONES)
    check_same(got, want)
    assert len(got[0]["types"]) == 60 and got[0]["capacity_type"] == "on-demand"
    assert got[1]["capacity_type"] == "spot" and got[1]["rejected_spot"] > 0
    assert any("metal" in catalog[t].name for t in got[2]["types"])
    assert not any("metal" in catalog[t].name for t in got[3]["types"]) and got[3]["rejected_exotic"] > 0
