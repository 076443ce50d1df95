"""Device path (libkp.so on the MI355X) vs the CPU oracle on identical inputs — bit-exact.

Compared: every pod's placement (NodeClaim creation index / existing node / error) and every NodeClaim's
NodePool, pod list in add order, and instance-type options after OrderByPrice + Truncate(100).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def canon(r):
    return [(n["nodepool"], n["pods"], n["options"], n["n_remaining"], n["requirements"]) for n in r["nodeclaims"]]


def check_same(got, want):
    diff = np.nonzero(got["placement"] != want["placement"])[0]
    assert len(diff) == 0, f"{len(diff)} placements differ, first pod {diff[:5]}: " \
                           f"{got['placement'][diff[:5]]} vs {want['placement'][diff[:5]]}"
    g, w = canon(got), canon(want)
    assert len(g) == len(w)
    for i, (a, b) in enumerate(zip(g, w)):
        assert a == b, f"NodeClaim {i} differs: {a[:2]} {a[3:]} vs {b[:2]} {b[3:]}"


def run_both(ctx, prob):
    import kpamd
    from oracle import pyoracle
    got = kpamd.Scheduler(ctx, prob).solve()
    want = pyoracle.solve(prob)
    return got, want


def test_config2_small(ctx, catalog):
    from kpamd import synth
    got, want = run_both(ctx, synth.config2(catalog, n_pods=400, seed=7))
    check_same(got, want)


def test_config1(ctx, catalog):
    from kpamd import synth
    got, want = run_both(ctx, synth.config1(catalog, n_pods=1000, seed=1))
    check_same(got, want)
    assert len(got["nodeclaims"]) > 0


@pytest.mark.parametrize("seed", range(12))
def test_random_scenarios(ctx, catalog, seed):
    from kpamd import synth
    prob = synth.random_problem(catalog, seed, n_types=150, n_pods=250, n_pools=3,
                                n_existing=[0, 5, 40][seed % 3], n_shapes=20)
    got, want = run_both(ctx, prob)
    check_same(got, want)


@pytest.mark.parametrize("seed,n_catalogs", [(100, 3), (105, 10)])
def test_multi_catalog(ctx, catalog, seed, n_catalogs):
    """Pools on different catalogues (GetInstanceTypes per NodeClass): per-catalogue Fits thresholds, PVP rows
    and offering classes, including catalogue ids >= 8 (no LDS pointer slot)."""
    from kpamd import synth
    prob = synth.random_problem(catalog, seed, n_types=150, n_pods=300, n_pools=max(3, n_catalogs),
                                n_existing=5, n_shapes=20, n_catalogs=n_catalogs)
    got, want = run_both(ctx, prob)
    check_same(got, want)
    assert len({n["nodepool"] for n in got["nodeclaims"]}) > 1


def test_config5_scaled(ctx, catalog):
    from kpamd import synth
    got, want = run_both(ctx, synth.config5(catalog, n_pods=3000, seed=5))
    check_same(got, want)


def test_config2_medium(ctx, catalog):
    from kpamd import synth
    got, want = run_both(ctx, synth.config2(catalog, n_pods=3000, seed=2))
    check_same(got, want)


@pytest.mark.parametrize("n_types", [37, 919])
def test_feasibility_kernel_vs_oracle(ctx, catalog, n_types):
    """CompatibleAvailableFilter for randomized (requirements, requests) rows: one partial 64-type tile (37) and
    the full catalogue (15 tiles: two lane batches of the kernel)."""
    import kpamd
    from kpamd import synth
    from oracle import pyoracle
    prob = synth.random_problem(catalog, 99, n_types=n_types, n_pods=10, n_shapes=40)
    rng = np.random.default_rng(3)
    queries = []
    for sh in prob.shapes:
        reqs = [r for t in sh.required_terms[:1] for r in t] + [(k, "In", [v]) for k, v in sh.node_selector.items()]
        queries.append((reqs, sh.requests))
    queries.append(([("karpenter.k8s.aws/instance-cpu", "Gt", ["15"]), ("kubernetes.io/arch", "NotIn", ["arm64"])],
                    {"cpu": 8000, "memory": 1 << 40}))
    cat = kpamd.Catalog(ctx, prob.catalogs[0])
    kept, cheapest, _ = kpamd.compatible_available_filter(ctx, cat, queries)
    for qi, (reqs, rq) in enumerate(queries):
        want_k, want_c = pyoracle.compatible_available_filter(prob.catalogs[0], reqs, rq)
        assert (kept[qi] == want_k).all(), f"query {qi}"
        np.testing.assert_array_equal(cheapest[qi][want_k], want_c[want_k])


def test_sort_spill_to_global(ctx, catalog, ov):
    """newNodeClaims order spills from LDS to global memory past the LDS capacity (forced small here)."""
    from kpamd import synth
    ov(sort_capacity=5)
    got, want = run_both(ctx, synth.config2(catalog, n_pods=2500, seed=11))
    check_same(got, want)
    assert len(got["nodeclaims"]) > 5


def test_repeated_runs_identical(ctx, catalog):
    """kp_solve_run restores all mutable device state: repeated runs of one plan give identical results."""
    import kpamd
    from kpamd import synth
    prob = synth.random_problem(catalog, 5, n_types=150, n_pods=250, n_existing=40, n_shapes=20)
    plan = kpamd.Scheduler(ctx, prob).prepare()
    r1, r2 = plan.run(), plan.run()
    plan.close()
    check_same(r1, r2)


def test_config2_many_nodeclaims(ctx, catalog):
    """>= 50 NodeClaims: exercises the ninther choosePivot / partialInsertionSort fast path of the
    device's sort.Slice replay against the oracle's literal pdqsort."""
    from kpamd import synth
    got, want = run_both(ctx, synth.config2(catalog, n_pods=12000, seed=2))
    check_same(got, want)
    assert len(got["nodeclaims"]) >= 50


def test_config5_many_pools(ctx, catalog):
    from kpamd import synth
    got, want = run_both(ctx, synth.config5(catalog, n_pods=6000, seed=5))
    check_same(got, want)


def test_filter_plan_pod_rows(ctx, catalog):
    """kp_filter_prepare/run over per-pod rows (the bench's feasibility leg) == the oracle, row by row."""
    import kpamd
    from kpamd import synth
    from oracle import pyoracle
    prob = synth.config2(catalog, n_pods=300, seed=9)
    queries = kpamd.pod_queries(prob)
    cat = kpamd.Catalog(ctx, catalog)
    fp = kpamd.FilterPlan(ctx, cat, queries, cheapest=True)
    kept, cheapest, st = fp.run(read=True)
    fp.close()
    assert st["attempts"] == len(queries) * len(catalog)
    seen = {}
    for qi, (reqs, rq) in enumerate(queries):
        key = int(prob.pod_shape[qi])
        if key not in seen:
            seen[key] = pyoracle.compatible_available_filter(catalog, reqs, rq)
        want_k, want_c = seen[key]
        assert (kept[qi] == want_k).all(), f"row {qi}"
        np.testing.assert_array_equal(cheapest[qi][want_k], want_c[want_k])


def test_feasibility_lds_staged_equals_global(ctx, catalog, ov):
    """The bitset kernels (feasibility_quad_kernel, four rows per wave, at this catalogue size; feasibility_bits_kernel,
    kp_overrides.feasibility_kernel 2) == feasibility_kernel (per-type global gathers, feasibility_kernel 1) bit for bit on pairwise-distinct
    rows (the bench's roofline leg: Gt/Lt bounds, NotIn, zones, capacity types; a row count that leaves the last quad
    partial), and == the oracle on a sample of rows."""
    import kpamd
    from kpamd import synth
    from oracle import pyoracle
    queries = synth.distinct_queries(catalog, 3001)
    cat = kpamd.Catalog(ctx, catalog)

    def run(qs, kernel=0):
        ov(feasibility_kernel=kernel)
        fp = kpamd.FilterPlan(ctx, cat, qs, cheapest=True)
        try:
            k, c, _ = fp.run(read=True)
        finally:
            fp.close()
        return k, c
    try:
        k1, c1 = run(queries)
        k2, c2 = run(queries, 1)
        k3, c3 = run(queries, 2)
        for nq in (1, 2, 3, 5):  # partial quads only
            ka, ca = run(queries[:nq])
            kb, cb = run(queries[:nq], 2)
            assert (ka == kb).all() and (ka == k1[:nq]).all(), nq
            np.testing.assert_array_equal(ca, cb)
    finally:
        cat.close()
    assert (k1 == k2).all() and (k1 == k3).all()
    np.testing.assert_array_equal(c1, c2)
    np.testing.assert_array_equal(c1, c3)
    assert k1.any() and not k1.all()
    for qi in range(0, len(queries), 97):
        want_k, want_c = pyoracle.compatible_available_filter(catalog, *queries[qi])
        assert (k1[qi] == want_k).all(), f"row {qi}"
        np.testing.assert_array_equal(c1[qi][want_k], want_c[want_k])


@pytest.mark.parametrize("n_pods", [3_000, 12_000])
def test_config2_burst(ctx, catalog, n_pods):
    """config 2 with ReplicaSet bursts (long same-shape-level runs onto one NodeClaim)."""
    from kpamd import synth
    got, want = run_both(ctx, synth.config2(catalog, n_pods=n_pods, seed=5, burst=True))
    check_same(got, want)


@pytest.mark.gpu
@pytest.mark.parametrize("kernel", [0, 2, 1])
def test_filter_compact_equals_expanded(ctx, catalog, ov, kernel):
    """KP_FILTER_COMPACT (ABI v11): the mask and each row's compatible offering classes; min over those classes of
    kp_filter_class_prices equals kp_filter_run's cheapest-price rows bit for bit, on every kernel (quad, one-row,
    per-type), including after an ICE refresh (R:pkg/providers/instance/filter/filter.go:39-64)."""
    import copy
    import kpamd
    from kpamd import synth
    ov(feasibility_kernel=kernel)
    queries = synth.distinct_queries(catalog, 1001)
    its = copy.deepcopy(catalog)
    cat = kpamd.Catalog(ctx, its, seqnum=1)
    fe = kpamd.FilterPlan(ctx, cat, queries, cheapest=True)
    fc = kpamd.FilterPlan(ctx, cat, queries, cheapest="compact")
    for step in range(2):
        k1, c1, _ = fe.run(read=True)
        k2, cls, _ = fc.run_compact(read=True)
        assert (k1 == k2).all()
        c2 = kpamd.FilterPlan.cheapest_from_compact(cls, fc.class_prices())
        np.testing.assert_array_equal(c1, c2)  # every type, its mask bit set or not (kp_abi.h)
        if step == 0:  # ICE marks: both plans refreshed in place
            cat.update_offerings([(t, "spot", "test-zone-1a", False) for t in range(0, len(catalog), 3)], seqnum=2)
            with pytest.raises(kpamd.KPError):  # the class prices of a stale plan are refused until the refresh
                fc.class_prices()
            fe.refresh(cat)
            fc.refresh(cat)
    with pytest.raises(kpamd.KPError):
        fe.run_compact(read=True)  # prepared without KP_FILTER_COMPACT
    fe.close()
    fc.close()
    cat.close()
