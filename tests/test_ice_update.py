"""ICE / price updates on a resident catalogue (kp_catalog_update_offerings, kp_filter_refresh).

Reference: UnavailableOfferings.MarkUnavailable bumps SeqNum (R:pkg/cache/unavailableofferings.go:66-92), which
changes the offering cache key (R:pkg/providers/instancetype/offering/offering.go:189-207) so InjectOfferings
rebuilds every offering with Available = !ICE && hasPrice && zone offered (R:offering.go:115-147). The expected
state after an update is therefore a catalogue built from scratch with the same ICE set
(`catalog.build_catalog(unavailable=...)`, the restatement of createOfferings); the device plan refreshed in place
must give bit-identical filter results to a plan prepared on that rebuilt catalogue.
"""
import copy
import ctypes as C
import math

import numpy as np
import pytest

# (capacity type, type index, zone) marks; type indices into the 919-type catalogue
MARKS = [("spot", 0, "test-zone-1a"), ("on-demand", 0, "test-zone-1b"), ("spot", 5, "test-zone-1c"),
         ("on-demand", 17, "test-zone-1a"), ("spot", 17, "test-zone-1a"), ("on-demand", 300, "test-zone-1c"),
         ("spot", 700, "test-zone-1b"), ("on-demand", 900, "test-zone-1a"), ("spot", 900, "test-zone-1a")]


def _host_catalog(lib, its):
    from kpamd import abi
    arena = abi.Arena()
    h = C.c_void_p()
    assert lib.kp_catalog_upload(None, C.byref(arena.catalog_desc(its)), 7, C.byref(h)) == 0
    return h, arena


def _updates(marks, avail=False, price=None):
    from kpamd import abi
    ups = [abi.OfferingUpdate(t, 1 if avail else 0, ct.encode(), z.encode(), math.nan if price is None else price)
           for ct, t, z in marks]
    return (abi.OfferingUpdate * len(ups))(*ups), len(ups)


def test_update_struct_layout():
    from kpamd import abi
    assert C.sizeof(abi.OfferingUpdate) == 4 + 4 + 8 + 8 + 8 + 8 + 4 + 4


def test_update_host_catalogue_and_seqnum(lib, catalog):
    h, _ = _host_catalog(lib, catalog)
    try:
        arr, n = _updates(MARKS)
        assert lib.kp_catalog_update_offerings(h, arr, n, 8) == 0
        assert lib.kp_catalog_seqnum(h) == 8
        assert lib.kp_catalog_update_offerings(h, arr, 0, 9) == 0  # empty update still bumps the seqnum
        assert lib.kp_catalog_seqnum(h) == 9
    finally:
        lib.kp_catalog_destroy(h)


@pytest.mark.parametrize("bad", [("spot", 919, "test-zone-1a"), ("spot", 3, "no-such-zone"),
                                 ("reserved", 3, "test-zone-1a")])
def test_update_rejects_unknown_offering_all_or_nothing(lib, catalog, bad):
    import kpamd
    h, _ = _host_catalog(lib, catalog)
    try:
        arr, n = _updates(MARKS[:2] + [bad])
        assert lib.kp_catalog_update_offerings(h, arr, n, 8) == kpamd.abi.KP_E_INVAL
        assert lib.kp_catalog_seqnum(h) == 7  # nothing applied
    finally:
        lib.kp_catalog_destroy(h)


def test_update_reserved_capacity_zero_cannot_be_available(lib):
    """R:offering.go:178: a reserved offering's Available is ReservationCapacity != 0 && zone in itZones, so an update
    that sets capacity 0 while marking it available is refused (all or nothing); capacity 0 + unavailable applies."""
    import kpamd
    from kpamd import abi, catalog as catmod
    rows = [r for r in catmod.load_ec2_table() if r["name"] in ("m5.large", "c5.xlarge")]
    crs = [catmod.CapacityReservation("cr-1", "m5.large", "test-zone-1a", available_count=3)]
    its = catmod.build_catalog(lib, rows=rows, capacity_reservations=crs)
    t = next(i for i, it in enumerate(its) if it.name == "m5.large")
    h, _ = _host_catalog(lib, its)
    try:
        def up(avail, cap):
            return (abi.OfferingUpdate * 1)(abi.OfferingUpdate(t, avail, b"reserved", b"test-zone-1a", math.nan, b"cr-1",
                                                                cap, 0))
        assert lib.kp_catalog_update_offerings(h, up(1, 0), 1, 8) == kpamd.abi.KP_E_INVAL
        assert lib.kp_catalog_seqnum(h) == 7
        assert lib.kp_catalog_update_offerings(h, up(0, 0), 1, 8) == 0
        assert lib.kp_catalog_update_offerings(h, up(1, 2), 1, 9) == 0
        assert lib.kp_catalog_seqnum(h) == 9
    finally:
        lib.kp_catalog_destroy(h)


def test_oracle_ice_marks_equal_rebuilt_catalogue(lib, catalog):
    """The update semantics (flip Available of the named offerings) == createOfferings with the ICE set."""
    from kpamd import catalog as kc
    from oracle import pyoracle
    names = [it.name for it in catalog]
    rebuilt = kc.build_catalog(lib, unavailable=frozenset((ct, names[t], z) for ct, t, z in MARKS))
    flipped = copy.deepcopy(catalog)
    for ct, t, z in MARKS:
        for o in flipped[t].offerings:
            if o.capacity_type == ct and o.zone == z:
                o.available = False
    for a, b in zip(rebuilt, flipped):
        assert [(o.capacity_type, o.zone, o.price, o.available) for o in a.offerings] == \
               [(o.capacity_type, o.zone, o.price, o.available) for o in b.offerings]
    reqs = [("topology.kubernetes.io/zone", "In", ["test-zone-1a"])]
    k1, c1 = pyoracle.compatible_available_filter(rebuilt, reqs, {"cpu": 100})
    k2, c2 = pyoracle.compatible_available_filter(flipped, reqs, {"cpu": 100})
    assert (k1 == k2).all() and not k1[17]  # both zone-1a offerings of type 17 are ICE'd
    np.testing.assert_array_equal(c1[k1], c2[k2])


@pytest.mark.gpu
def test_filter_refresh_equals_rebuilt_plan(ctx, lib, catalog):
    """Resident plan + ICE marks + kp_filter_refresh == plan prepared on the rebuilt catalogue, and both == the
    oracle; then un-marking with new prices restores / reprices exactly."""
    import kpamd
    from kpamd import catalog as kc
    from kpamd import synth
    from oracle import pyoracle
    prob = synth.config2(catalog, n_pods=400, seed=21)
    queries = kpamd.pod_queries(prob)
    queries.append(([("topology.kubernetes.io/zone", "In", ["test-zone-1a"])], {"cpu": 100}))
    its = copy.deepcopy(catalog)
    cat = kpamd.Catalog(ctx, its, seqnum=1)
    fp = kpamd.FilterPlan(ctx, cat, queries, cheapest=True)
    k0, c0, _ = fp.run(read=True)
    cat.update_offerings([(t, ct, z, False) for ct, t, z in MARKS], seqnum=2)
    assert cat.seqnum() == 2
    with pytest.raises(kpamd.KPError, match="stale plan"):  # offerings changed: the plan must be refreshed first
        fp.run(read=True)
    fp.refresh(cat)
    k1, c1, _ = fp.run(read=True)
    names = [it.name for it in catalog]
    rebuilt = kc.build_catalog(lib, unavailable=frozenset((ct, names[t], z) for ct, t, z in MARKS))
    cat2 = kpamd.Catalog(ctx, rebuilt)
    fp2 = kpamd.FilterPlan(ctx, cat2, queries, cheapest=True)
    k2, c2, _ = fp2.run(read=True)
    assert (k1 == k2).all()
    np.testing.assert_array_equal(c1, c2)
    assert not (k0 == k1).all()  # the marks changed something (query -1 lost type 17)
    want_k, want_c = pyoracle.compatible_available_filter(rebuilt, queries[-1][0], queries[-1][1])
    assert (k1[-1] == want_k).all()
    np.testing.assert_array_equal(c1[-1][want_k], want_c[want_k])
    # clear the marks and reprice one offering: the refreshed plan follows the new prices
    cat.update_offerings([(t, ct, z, True) for ct, t, z in MARKS] + [(5, "spot", "test-zone-1c", True, 0.0001)],
                         seqnum=3)
    fp.refresh(cat)
    k3, c3, _ = fp.run(read=True)
    assert (k3 == k0).all()
    want_k, want_c = pyoracle.compatible_available_filter(its, queries[0][0], queries[0][1])
    assert (k3[0] == want_k).all()
    np.testing.assert_array_equal(c3[0][want_k], want_c[want_k])
    # a plan refreshes only from the catalogue it was prepared on
    with pytest.raises(kpamd.KPError):
        fp.refresh(cat2)
    for x in (fp, fp2, cat, cat2):
        x.close()


@pytest.mark.gpu
def test_launch_refresh_equals_rebuilt_catalogue(ctx, lib, catalog):
    """Launch-side selection after ICE marks (the reference's ICE fallback, R:pkg/providers/instancetype/
    suite_test.go:2059-2092): a resident launch plan refreshed in place == the oracle on the rebuilt catalogue."""
    import kpamd
    from kpamd import catalog as kc
    from kpamd import synth
    from oracle import pyoracle
    marks = [("spot", t, "test-zone-1a") for t in range(0, len(catalog), 2)] + \
            [("on-demand", t, "test-zone-1b") for t in range(0, len(catalog), 3)]
    reqs = synth.random_launch_requests(catalog, 200, seed=311)
    its = copy.deepcopy(catalog)
    cat = kpamd.Catalog(ctx, its, seqnum=1)
    plan = kpamd.LaunchPlan(ctx, cat, reqs, kc.ZONES)
    before, _ = plan.run(read=True)
    cat.update_offerings([(t, ct, z, False) for ct, t, z in marks], seqnum=2)
    with pytest.raises(kpamd.KPError, match="stale plan"):
        plan.run(read=True)
    plan.refresh(cat)
    got, _ = plan.run(read=True)
    names = [it.name for it in catalog]
    rebuilt = kc.build_catalog(lib, unavailable=frozenset((ct, names[t], z) for ct, t, z in marks))
    want = pyoracle.launch_select(rebuilt, reqs, kc.ZONES, max_types=60)
    assert len(got) == len(want)
    for i, (g, w) in enumerate(zip(got, want)):
        assert g == w, f"request {i}: device {g} vs oracle {w}"
    assert got != before  # the marks moved some launches (overrides or capacity type)
    plan.close()
    cat.close()


@pytest.mark.gpu
def test_solve_catalogue_resident_across_seqnums(ctx, lib, catalog):
    """The Solve's compiled catalogue half stays resident in the kp_ctx across Solves (same catalogue identity,
    seqnum and NodePools: catalog_cached = 1) and has its offerings re-applied in place when an ICE mark bumps the
    seqnum (catalog_refreshed = 1)
    (R:pkg/providers/instancetype/instancetype.go:225-237 cacheKey; R:pkg/cache/unavailableofferings.go:66-92);
    every Solve equals the oracle on the catalogue as it is at that moment."""
    import kpamd
    from kpamd import catalog as kc
    from kpamd import synth
    from oracle import pyoracle
    its = copy.deepcopy(catalog)
    cat = kpamd.Catalog(ctx, its, seqnum=1)
    prob = synth.config2(its, n_pods=600, seed=23)
    sched = kpamd.Scheduler(ctx, prob, catalogs=[cat])
    first = sched.solve()
    second = sched.solve()
    assert second["stats"]["catalog_cached"] == 1
    want = pyoracle.solve(prob)
    for got in (first, second):
        assert (got["placement"] == want["placement"]).all()
        assert [(n["nodepool"], n["pods"], n["options"]) for n in got["nodeclaims"]] == \
            [(n["nodepool"], n["pods"], n["options"]) for n in want["nodeclaims"]]
    marks = [("spot", t, z) for t in range(0, len(its), 2) for z in kc.ZONES[:2]] + \
            [("on-demand", t, "test-zone-1a") for t in range(len(its))]
    cat.update_offerings([(t, ct, z, False) for ct, t, z in marks], seqnum=2)
    third = sched.solve()
    assert third["stats"]["catalog_cached"] == 1 and third["stats"]["catalog_refreshed"] == 1
    names = [it.name for it in catalog]
    rebuilt = kc.build_catalog(lib, unavailable=frozenset((ct, names[t], z) for ct, t, z in marks))
    want = pyoracle.solve(synth.config2(rebuilt, n_pods=600, seed=23))
    assert (third["placement"] == want["placement"]).all()
    assert [(n["nodepool"], n["pods"], n["options"]) for n in third["nodeclaims"]] == \
        [(n["nodepool"], n["pods"], n["options"]) for n in want["nodeclaims"]]
    assert [n["options"] for n in third["nodeclaims"]] != [n["options"] for n in first["nodeclaims"]]
    cat.close()


def _marks(its):
    from kpamd import catalog as kc
    return [("spot", t, z) for t in range(0, len(its), 2) for z in kc.ZONES[:2]] + \
        [("on-demand", t, "test-zone-1a") for t in range(len(its))] + [("on-demand", t, "test-zone-1b") for t in range(0, len(its), 3)]


def _canon(res):
    return (res["placement"].tolist(), [(n["nodepool"], n["pods"], n["options"], n["n_remaining"], n["requirements"])
                                        for n in res["nodeclaims"]])


@pytest.mark.gpu
def test_solve_plan_refresh_equals_rebuilt_catalogue(ctx, lib, catalog):
    """kp_solve_refresh (R:pkg/cache/unavailableofferings.go:66-92 SeqNum): a prepared plan refuses to run once its
    catalogue's seqnum moved; refreshed in place (offering masks, class prices, template options, the per-Solve
    template table) it equals the oracle on a catalogue rebuilt with those offerings unavailable, and a second
    Solve on the ctx reuses the refreshed half."""
    import kpamd
    from kpamd import catalog as kc
    from kpamd import synth
    from oracle import pyoracle
    its = copy.deepcopy(catalog)
    cat = kpamd.Catalog(ctx, its, seqnum=1)
    prob = synth.config5(its, n_pods=3000)
    sched = kpamd.Scheduler(ctx, prob, catalogs=[cat])
    plan = sched.prepare()
    before = plan.run()
    marks = _marks(its)
    cat.update_offerings([(t, ct, z, False) for ct, t, z in marks], seqnum=2)
    with pytest.raises(kpamd.KPError) as e:
        plan.run()
    assert e.value.code == kpamd.abi.KP_E_INVAL
    plan.refresh()
    after = plan.run()
    plan.close()
    names = [it.name for it in catalog]
    rebuilt = kc.build_catalog(lib, unavailable=frozenset((ct, names[t], z) for ct, t, z in marks))
    want = pyoracle.solve(synth.config5(rebuilt, n_pods=3000))
    assert _canon(after) == _canon(want)
    assert _canon(after) != _canon(before)
    again = sched.solve()
    assert again["stats"]["catalog_cached"] == 1 and again["stats"]["catalog_refreshed"] == 0
    assert _canon(again) == _canon(want)
    cat.close()


@pytest.mark.gpu
def test_cluster_plan_refresh_equals_rebuilt_catalogue(ctx, lib, catalog):
    """kp_cluster_refresh: a resident consolidation snapshot after ICE marks equals the oracle's
    computeConsolidation on the rebuilt catalogue; before the refresh it refuses to simulate."""
    import kpamd
    from kpamd import catalog as kc
    from kpamd import synth
    from oracle import pyoracle
    its = copy.deepcopy(catalog)
    cl = synth.config4(its, n_nodes=150, seed=4)
    cat = kpamd.Catalog(ctx, cl.catalogs[0], seqnum=1)
    plan = kpamd.ClusterPlan(ctx, cl, catalogs=[cat])
    subs = synth.consolidation_subsets(cl, 60, seed=5)
    before, _ = plan.simulate(subs)
    marks = _marks(its)
    cat.update_offerings([(t, ct, z, False) for ct, t, z in marks], seqnum=2)
    with pytest.raises(kpamd.KPError):
        plan.simulate(subs)
    plan.refresh()
    after, _ = plan.simulate(subs)
    plan.close()
    cat.close()
    names = [it.name for it in catalog]
    rebuilt = kc.build_catalog(lib, unavailable=frozenset((ct, names[t], z) for ct, t, z in marks))
    cl2 = copy.copy(cl)
    cl2.catalogs = [rebuilt]
    want, _ = pyoracle.simulate_batch(cl2, subs)
    fields = ("decision", "nodepool", "candidate_price", "replacement_price", "savings", "n_options", "n_pods")
    assert [tuple(r[f] for f in fields) for r in after] == [tuple(r[f] for f in fields) for r in want]
    assert [tuple(r[f] for f in fields) for r in after] != [tuple(r[f] for f in fields) for r in before]
