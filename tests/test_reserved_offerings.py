"""Reserved (capacity-reservation) offerings on the launch path.

Oracle pins: the CapacityReservationType / CapacityBlock / ReservedOffering filter cases of
R:pkg/providers/instance/filter/filter_test.go:130-396, transcribed as data below (kept / rejected names and the
offerings a kept type retains). Device: kp_launch_select (launch_kernel) against the oracle's launch selection,
bit-exact, on catalogues carrying reservations (R:pkg/providers/instancetype/offering/offering.go:151-186 builds
them: capacity type reserved, the reservation id and type labels, ReservationCapacity), gpu-marked.
"""
import dataclasses

import numpy as np
import pytest

from kpamd.model import InstanceType, Offering

CT = "karpenter.sh/capacity-type"
Z = "topology.kubernetes.io/zone"
K = "karpenter.k8s.aws/"
RTYPES = ["default", "capacity-block"]  # v1.CapacityReservationType("").Values(), priority order


def off(ct, avail, price=0.0, zone=None, rt=None, rid=None, cap=0):
    return Offering(ct, zone, None, float(price), bool(avail), rid, rt, int(cap))


def it(name, *offs):
    return InstanceType(name, [], {}, {}, list(offs))


def run(which, types, reqs):
    from oracle import pyoracle
    kept, offs = pyoracle.reservation_filter(types, reqs, which)
    return ({t.name for t, k in zip(types, kept) if k}, {t.name for t, k in zip(types, kept) if not k},
            {t.name: [t.offerings[j] for j in o] for t, k, o in zip(types, kept, offs) if k})


# ---- CapacityReservationTypeFilter (R:filter_test.go:130-255) ----------------------------------------------
@pytest.mark.parametrize("sel", RTYPES)
def test_crt_prioritizes_cheapest_type(sel):
    kept_types = [it(f"cheap-instance-{sel}", off("reserved", True, 5.0, "zone-1a", rt=sel)),
                  it(f"expensive-instance-{sel}", off("reserved", True, 10.0, "zone-1a", rt=sel))]
    rejected = [it(f"expensive-instance-{t}", off("reserved", True, 10.0, "zone-1a", rt=t),
                   off("reserved", False, 1.0, "zone-1a", rt=t), off("reserved", True, 1.0, "zone-1b", rt=t))
                for t in RTYPES if t != sel]
    kept, rej, _ = run("type", kept_types + rejected, [(CT, "In", ["reserved"]), (Z, "In", ["zone-1a"])])
    assert kept == {t.name for t in kept_types} and rej == {t.name for t in rejected}


def test_crt_breaks_ties_by_priority():
    kept, rej, _ = run("type", [it("default", off("reserved", True, 5.0, rt="default")),
                                it("capacity-block", off("reserved", True, 5.0, rt="capacity-block"))],
                       [(CT, "In", ["reserved"])])
    assert kept == {"default"} and rej == {"capacity-block"}


@pytest.mark.parametrize("sel", RTYPES)
def test_crt_removes_other_type_offerings(sel):
    types = [it("pin-instance", off("reserved", True, 1.0, rt=sel)),
             it("filter-instance", *[off("reserved", True, 5.0, rt=t) for t in RTYPES])]
    kept, rej, offs = run("type", types, [(CT, "In", ["reserved"])])
    assert kept == {"pin-instance", "filter-instance"} and not rej
    for name in kept:
        assert len(offs[name]) == 1
        assert offs[name][0].capacity_type == "reserved" and offs[name][0].reservation_type == sel


def test_crt_not_compatible_with_reserved():
    types = [it(f"{t}-instance", off("on-demand", True), off("reserved", True, 1.0, rt=t)) for t in RTYPES]
    kept, rej, offs = run("type", types, [(CT, "NotIn", ["reserved"])])
    assert kept == {t.name for t in types} and not rej
    assert all(len(o) == 2 for o in offs.values())


# ---- CapacityBlockFilter (R:filter_test.go:257-320) ----------------------------------------------------------
def test_cb_selects_cheapest_capacity_block():
    types = [it("cheap-instance", off("reserved", True, 1.0, rt="capacity-block"), off("reserved", True, 10.0, rt="capacity-block")),
             it("expensive-instance", off("reserved", True, 2.0, rt="capacity-block"),
                off("reserved", True, 10.0, rt="capacity-block"))]
    kept, rej, offs = run("block", types, [(CT, "Exists", [])])
    assert kept == {"cheap-instance"} and rej == {"expensive-instance"}
    assert [o.price for o in offs["cheap-instance"]] == [1.0]


def test_cb_ignores_other_reservation_types():
    types = [it("cheap-instance", off("reserved", True, 1.0, rt="default"), off("reserved", True, 10.0, rt="default")),
             it("expensive-instance", off("reserved", True, 2.0, rt="default"), off("reserved", True, 10.0, rt="default"))]
    kept, rej, _ = run("block", types, [(CT, "Exists", [])])
    assert kept == {"cheap-instance", "expensive-instance"} and not rej


def test_cb_not_compatible_with_reserved():
    types = [it("cheap-instance", off("reserved", True, 1.0, rt="capacity-block"), off("on-demand", True, 1.0, rt="capacity-block")),
             it("expensive-instance", off("reserved", True, 2.0, rt="capacity-block"),
                off("on-demand", True, 2.0, rt="capacity-block"))]
    kept, rej, _ = run("block", types, [(CT, "NotIn", ["reserved"])])
    assert kept == {"cheap-instance", "expensive-instance"} and not rej


# ---- ReservedOfferingFilter (R:filter_test.go:322-396) -------------------------------------------------------
def test_rof_no_available_reserved_offerings():
    types = [it("non-reserved-instance", off("on-demand", True), off("spot", True)),
             it("reserved-instance", off("on-demand", True), off("spot", True), off("reserved", False))]
    kept, rej, _ = run("offering", types, [(CT, "Exists", [])])
    assert kept == {"non-reserved-instance", "reserved-instance"} and not rej


def test_rof_one_offering_per_zone():
    types = [it("non-reserved-instance", off("on-demand", True), off("spot", True)),
             it("reserved-instance-a", off("on-demand", True), off("spot", True),
                off("reserved", True, zone="1", rid="kept", cap=5), off("reserved", True, zone="2", rid="kept", cap=6),
                off("reserved", True, zone="2", rid="rejected", cap=5)),
             it("reserved-instance-b", off("on-demand", True), off("spot", True),
                off("reserved", True, zone="1", rid="kept", cap=1), off("reserved", False, zone="1", rid="rejected", cap=2))]
    kept, rej, offs = run("offering", types, [(CT, "Exists", [])])
    assert kept == {"reserved-instance-a", "reserved-instance-b"} and rej == {"non-reserved-instance"}
    assert len(offs["reserved-instance-a"]) == 2
    assert all(o.reservation_id == "kept" for v in offs.values() for o in v)


def test_rof_not_compatible_with_reserved():
    types = [it("non-reserved-instance", off("on-demand", True), off("spot", True)),
             it("reserved-instance", off("on-demand", True), off("spot", True), off("reserved", True, zone="1"))]
    kept, rej, offs = run("offering", types, [(CT, "NotIn", ["reserved"])])
    assert kept == {"non-reserved-instance", "reserved-instance"} and not rej
    assert sorted(len(o) for o in offs.values()) == [2, 3]


# ---- launch-level behaviour (oracle) ---------------------------------------------------------------------------
def test_launch_prefers_reserved_then_reports_type():
    """getCapacityType: reserved first (R:instance.go:504-518); getCapacityReservationType on the kept slices;
    overrides only from the reserved offering ReservedOfferingFilter kept per zone."""
    from oracle import pyoracle
    types = [InstanceType("m5.large", [(CT, "In", ["on-demand", "spot", "reserved"])], {"cpu": 2000}, {},
                          [off("on-demand", True, 0.1, "zone-1a"), off("spot", True, 0.03, "zone-1a"),
                           off("reserved", True, 1e-8, "zone-1a", rt="default", rid="cr-a", cap=2),
                           off("reserved", True, 1e-8, "zone-1a", rt="default", rid="cr-b", cap=3)]),
             InstanceType("m5.xlarge", [(CT, "In", ["on-demand", "spot"])], {"cpu": 4000}, {},
                          [off("on-demand", True, 0.2, "zone-1a"), off("spot", True, 0.05, "zone-1a")])]
    reqs = [([(CT, "In", ["on-demand", "spot", "reserved"])], {"cpu": 1000}, [0, 1]),
            ([(CT, "In", ["on-demand", "spot"])], {"cpu": 1000}, [0, 1])]
    r = pyoracle.launch_select(types, reqs, ["zone-1a"])
    assert r[0]["capacity_type"] == "reserved" and r[0]["reservation_type"] == "default"
    assert r[0]["types"] == [0] and r[0]["rejected_reservation"] == 1
    assert r[0]["overrides"] == [(0, "zone-1a")]  # cr-b (capacity 3) only
    assert r[1]["capacity_type"] == "spot" and r[1]["reservation_type"] is None


# ---- device vs oracle ------------------------------------------------------------------------------------------
def reserved_catalogue(catalog, n_types, seed):
    """The first n_types docs types through kpamd.catalog.build_catalog with 18 random types holding 1-3 capacity
    reservations each (offering.go:151-186: price OD / 1e7, Available = count != 0, ReservationCapacity = count;
    types.go:172,223-232: the type's requirements gain reserved / the ids / the types). Every reservation is an
    offering class of its own: <= 54 of the device's 64 classes. `catalog` only fixes the library (lib)."""
    from kpamd import catalog as cmod
    import kpamd
    rng = np.random.default_rng(seed)
    rows = cmod.load_ec2_table()[:n_types]
    crs = []
    for i in sorted(rng.choice(n_types, size=18, replace=False).tolist()):
        for _ in range(int(rng.integers(1, 4))):
            crs.append(cmod.CapacityReservation(f"cr-{len(crs) + 1:05d}", rows[i]["name"], str(rng.choice(cmod.ZONES)),
                                                RTYPES[int(rng.random() < 0.3)], int(rng.choice([0, 1, 2, 5, 9]))))
    return cmod.build_catalog(kpamd.load_lib(), rows=rows, capacity_reservations=crs)


def test_catalogue_reservations_kat(catalog):
    """createOfferings / computeRequirements with reservations (R:offering.go:151-186, R:types.go:172,223-232)."""
    from kpamd import catalog as cmod
    import kpamd
    rows = [r for r in cmod.load_ec2_table() if r["name"] in ("m5.large", "c5.xlarge")]
    crs = [cmod.CapacityReservation("cr-1", "m5.large", cmod.ZONES[0], "default", 3),
           cmod.CapacityReservation("cr-2", "m5.large", cmod.ZONES[1], "capacity-block", 0)]
    cat = {t.name: t for t in cmod.build_catalog(kpamd.load_lib(), rows=rows, capacity_reservations=crs)}
    m5, c5 = cat["m5.large"], cat["c5.xlarge"]
    req = {r[0]: r for r in m5.requirements}
    assert req[CT][2] == ["on-demand", "spot", "reserved"]
    assert req[K + "capacity-reservation-id"] == (K + "capacity-reservation-id", "In", ["cr-1", "cr-2"])
    assert req[K + "capacity-reservation-type"][1:] == ("In", ["capacity-block", "default"])
    res = [o for o in m5.offerings if o.capacity_type == "reserved"]
    od = next(o.price for o in m5.offerings if o.capacity_type == "on-demand")
    assert [(o.reservation_id, o.zone, o.available, o.reservation_capacity) for o in res] == \
        [("cr-1", cmod.ZONES[0], True, 3), ("cr-2", cmod.ZONES[1], False, 0)]
    assert all(o.price == od / 10_000_000.0 for o in res)
    creq = {r[0]: r for r in c5.requirements}
    assert creq[CT][2] == ["on-demand", "spot"] and creq[K + "capacity-reservation-id"][1] == "DoesNotExist"
    assert not any(o.capacity_type == "reserved" for o in c5.offerings)


def reserved_requests(cat, n, seed):
    from kpamd import synth
    rng = np.random.default_rng(seed + 1)
    out = []
    for reqs, res, types in synth.random_launch_requests(cat, n, seed=seed):
        reqs = [r for r in reqs if r[0] != CT]
        k = rng.random()
        if k < 0.3:
            reqs.append((CT, "In", ["reserved"]))
        elif k < 0.55:
            reqs.append((CT, "In", ["reserved", "on-demand", "spot"]))
        elif k < 0.65:
            reqs.append((CT, "In", ["reserved", "spot"]))
        elif k < 0.75:
            reqs.append((CT, "NotIn", ["reserved"]))
        if rng.random() < 0.15:
            reqs.append((K + "capacity-reservation-type", "In", [str(rng.choice(RTYPES))]))
        if rng.random() < 0.05:
            reqs.append((K + "capacity-reservation-type", "DoesNotExist", []))
        out.append((reqs, res, types))
    return out


@pytest.mark.parametrize("seed", range(3))
def test_oracle_launch_random_reserved_smoke(catalog, seed):
    """CPU: the oracle runs the whole chain on reserved catalogues and picks reserved capacity somewhere."""
    from oracle import pyoracle
    from kpamd import catalog as cmod
    cat = reserved_catalogue(catalog, 300, seed)
    r = pyoracle.launch_select(cat, reserved_requests(cat, 80, 40 + seed), cmod.ZONES)
    cts = {x["capacity_type"] for x in r if x["status"] == 0}
    assert "reserved" in cts and ("on-demand" in cts or "spot" in cts)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(4))
def test_device_launch_reserved_matches_oracle(ctx, catalog, seed):
    import kpamd
    from kpamd import catalog as cmod
    from oracle import pyoracle
    cat = reserved_catalogue(catalog, 400 if seed < 2 else len(catalog), seed)
    reqs = reserved_requests(cat, 250, 40 + seed)
    zones = [cmod.ZONES, cmod.ZONES[:2], cmod.ZONES, cmod.ZONES[1:]][seed]
    ch = kpamd.Catalog(ctx, cat)
    plan = kpamd.LaunchPlan(ctx, ch, reqs, zones)
    got, _ = plan.run(read=True)
    plan.close()
    ch.close()
    want = pyoracle.launch_select(cat, reqs, zones)
    for i, (g, w) in enumerate(zip(got, want)):
        assert g == w, f"request {i}: device {g} vs oracle {w}"
    assert sum(g["capacity_type"] == "reserved" for g in got) > 0
    assert sum(g["rejected_reservation"] > 0 for g in got) > 0


def _cb_first_types():
    """The first type's first offering is a capacity block in a zone the request excludes: no reserved offering is
    compatible, yet CapacityBlockFilter's shouldFilter (R:filter.go:204-220) looks only at that first offering and the
    requirement admitting reserved, so it applies."""
    return [InstanceType("cb-first", [(CT, "In", ["on-demand", "reserved"])], {"cpu": 2000}, {},
                         [off("reserved", True, 0.5, "zone-1a", rt="capacity-block", rid="cr-cb", cap=1),
                          off("on-demand", True, 0.2, "zone-1b")]),
            InstanceType("plain", [(CT, "In", ["on-demand"])], {"cpu": 2000}, {}, [off("on-demand", True, 0.1, "zone-1b")])]


def test_oracle_capacity_block_without_compatible_reservation():
    kept, rej, offs = run("block", _cb_first_types(), [(CT, "In", ["on-demand", "reserved"]), (Z, "In", ["zone-1b"])])
    assert kept == {"cb-first"} and rej == {"plain"}
    assert [o.reservation_type for o in offs["cb-first"]] == ["capacity-block"]


@pytest.mark.gpu
def test_device_launch_capacity_block_without_compatible_reservation(ctx):
    import kpamd
    from oracle import pyoracle
    types = _cb_first_types()
    reqs = [([(CT, "In", ["on-demand", "reserved"]), (Z, "In", ["zone-1b"])], {"cpu": 1000}, [0, 1]),
            ([(CT, "In", ["on-demand"]), (Z, "In", ["zone-1b"])], {"cpu": 1000}, [0, 1])]
    ch = kpamd.Catalog(ctx, types)
    plan = kpamd.LaunchPlan(ctx, ch, reqs, ["zone-1a", "zone-1b"])
    got, _ = plan.run(read=True)
    plan.close()
    ch.close()
    want = pyoracle.launch_select(types, reqs, ["zone-1a", "zone-1b"])
    assert got == want
    assert got[0]["types"] == [0] and got[0]["rejected_reservation"] == 1 and len(got[1]["types"]) == 2


@pytest.mark.gpu
def test_device_launch_reserved_kat(ctx):
    import kpamd
    types = [InstanceType("m5.large", [(CT, "In", ["on-demand", "spot", "reserved"])], {"cpu": 2000}, {},
                          [off("on-demand", True, 0.1, "zone-1a"), off("spot", True, 0.03, "zone-1a"),
                           off("reserved", True, 1e-8, "zone-1a", rt="default", rid="cr-a", cap=2),
                           off("reserved", True, 1e-8, "zone-1a", rt="default", rid="cr-b", cap=3)]),
             InstanceType("m5.xlarge", [(CT, "In", ["on-demand", "spot"])], {"cpu": 4000}, {},
                          [off("on-demand", True, 0.2, "zone-1a"), off("spot", True, 0.05, "zone-1a")])]
    reqs = [([(CT, "In", ["on-demand", "spot", "reserved"])], {"cpu": 1000}, [0, 1]),
            ([(CT, "In", ["on-demand", "spot"])], {"cpu": 1000}, [0, 1])]
    ch = kpamd.Catalog(ctx, types)
    plan = kpamd.LaunchPlan(ctx, ch, reqs, ["zone-1a"])
    got, _ = plan.run(read=True)
    plan.close()
    ch.close()
    assert got[0]["capacity_type"] == "reserved" and got[0]["reservation_type"] == "default"
    assert got[0]["overrides"] == [(0, "zone-1a")] and got[0]["rejected_reservation"] == 1
    assert got[1]["capacity_type"] == "spot"


@pytest.mark.gpu
def test_cluster_over_reservations(ctx, catalog):
    """A consolidation cluster over a catalogue with reservation offerings (ABI v10) takes the general path, every
    simulation batched on the superset Solve with strict reservations; decisions equal the oracle's
    (tests/test_reserved_consolidation.py holds the design KATs)."""
    import kpamd
    from kpamd import synth
    from oracle import pyoracle
    cat = reserved_catalogue(catalog, 200, 0)
    cl = synth.random_cluster(cat, 0, n_nodes=10)
    subs = synth.consolidation_subsets(cl, 8, seed=3, max_size=5) + [[c] for c in cl.candidates[:5]]
    plan = kpamd.ClusterPlan(ctx, cl)
    try:
        got, st = plan.simulate(subs)
    finally:
        plan.close()
    assert st["phase_cycles"][0] == len(subs)
    want, _ = pyoracle.simulate_batch(cl, subs)
    assert [(g["decision"], g["savings"]) for g in got] == [(w["decision"], w["savings"]) for w in want]


@pytest.mark.gpu
def test_device_compatible_available_with_reservations(ctx, catalog):
    """CompatibleAvailableFilter rows over reservation classes (feasibility_kernel): kept masks and the cheapest
    compatible available price equal the oracle's, including queries pinning a reservation type or DoesNotExist."""
    import kpamd
    from oracle import pyoracle
    cat = reserved_catalogue(catalog, 300, 7)
    queries = [(r, q) for r, q, _ in reserved_requests(cat, 40, 77)]
    ch = kpamd.Catalog(ctx, cat)
    kept, cheapest, _ = kpamd.compatible_available_filter(ctx, ch, queries)
    ch.close()
    n_res_kept = 0
    for i, (r, q) in enumerate(queries):
        wk, wc = pyoracle.compatible_available_filter(cat, r, q)
        assert (kept[i] == wk).all(), f"query {i}"
        assert np.array_equal(np.where(wk, cheapest[i], 0), np.where(wk, wc, 0)), f"query {i}"
        if any(x == (CT, "In", ["reserved"]) for x in r):
            n_res_kept += int(wk.sum())
    assert n_res_kept > 0


@pytest.mark.gpu
def test_device_launch_reservation_updates_refresh(ctx, catalog):
    """Reservation ICE / capacity updates by id (kp_offering_update.reservation_id / reservation_capacity) on a
    prepared launch plan: kp_launch_refresh re-applies availability, prices and the capacity table; the result equals
    the oracle on the updated catalogue."""
    import kpamd
    from kpamd import catalog as cmod
    from oracle import pyoracle
    cat = reserved_catalogue(catalog, 400, 3)
    reqs = reserved_requests(cat, 150, 53)
    ch = kpamd.Catalog(ctx, cat)
    plan = kpamd.LaunchPlan(ctx, ch, reqs, cmod.ZONES)
    ups, k = [], 0
    for ti, t in enumerate(ch.instance_types):
        for o in t.offerings:
            if o.reservation_id:
                cap = [0, 7, 1][k % 3]
                k += 1
                ups.append((ti, "reserved", o.zone, cap != 0, None, o.reservation_id, cap))
    ch.update_offerings(ups, ch.seqnum() + 1)
    plan.refresh(ch)
    got, _ = plan.run(read=True)
    plan.close()
    want = pyoracle.launch_select(ch.instance_types, reqs, cmod.ZONES)
    ch.close()
    for i, (g, w) in enumerate(zip(got, want)):
        assert g == w, f"request {i}: device {g} vs oracle {w}"
    assert sum(g["capacity_type"] == "reserved" for g in got) > 0
