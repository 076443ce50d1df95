"""Capacity reservations inside Scheduler.Solve (ABI v9): upstream NodeClaim.reserveOfferings + ReservationManager.

Restated algorithm (oracle/oracle.cpp ReservationManager / Scheduler::ReserveOfferings; upstream karpenter
scheduling/nodeclaim.go and reservationmanager.go are not in the container):
  * the manager starts every reservation id at the least ReservationCapacity the NodePools' instance types report;
  * NodeClaim.Add, after filterInstanceTypesByRequirements, reserves every available reserved offering of a remaining type
    that is compatible with the NodeClaim's new requirements (Reserve is idempotent per hostname), and releases the ones it
    held that are no longer compatible;
  * strict mode (the provisioner's DisableReservedCapacityFallback) fails the Add when compatible reserved offerings exist
    but none could be reserved, or the NodeClaim held some and now holds none; such a pod is not relaxed;
  * FinalizeScheduling adds reservation-id In {held ids}, so the launch targets exactly the reservations counted.
The design is R:designs/odcr.md:248-256 ("count the number of simulated NodeClaims that might use the offering ... can't
simulate NodeClaims into particular offerings once they hit their cap"). Pinned end to end by the reference's own
scenarios R:pkg/cloudprovider/suite_test.go:1422-1505 (reserved-only NodePool: one NodeClaim, launched into the
reservation, available count 10 -> 9; the reservation-type selector picks that reservation's id and type); the capacity
cap and the release are the design's stated behaviour ("parity unpinned" beyond it). The device is checked against the
oracle on the same KATs and on randomized batches in both modes (-m gpu).
"""
import numpy as np
import pytest

CT = "karpenter.sh/capacity-type"
K = "karpenter.k8s.aws/"
RID = K + "capacity-reservation-id"
RT = K + "capacity-reservation-type"
RTYPES = ["default", "capacity-block"]
ZONE = "topology.kubernetes.io/zone"
IT = "node.kubernetes.io/instance-type"
STRICT, FALLBACK = 1, 0


def _rows(names):
    from kpamd import catalog as cmod
    table = {r["name"]: r for r in cmod.load_ec2_table()}
    return [table[n] for n in names]


def suite_catalogue(lib, count=10):
    """The suite's BeforeEach (R:pkg/cloudprovider/suite_test.go:1425-1446): one targeted reservation per reservation
    type for m5.large in test-zone-1a, each with 10 available instances, on the fake EC2 instance types."""
    from kpamd import catalog as cmod
    from scenarios import _fake_offering_zones
    names = sorted(_fake_offering_zones())
    crs = [cmod.CapacityReservation(f"cr-m5.large-1a-{rt}", "m5.large", "test-zone-1a", rt, count) for rt in RTYPES]
    return cmod.build_catalog(lib, rows=_rows(names), capacity_reservations=crs)


def reserved_pool(reqs=()):
    from kpamd.model import NodePool
    return NodePool("default", 0, 0, [(CT, "In", ["reserved"])] + list(reqs))


def problem(cat, pools, shapes, counts, mode):
    from kpamd.model import Problem
    from scenarios import pods_of
    s, c, u = pods_of(counts)
    return Problem([cat], pools, shapes, s, c, u, name="reserved", reserved_offering_mode=mode)


def solve(backend, prob, ctx=None):
    if backend == "device":
        import kpamd
        return kpamd.Scheduler(ctx, prob).solve()
    from oracle import pyoracle
    return pyoracle.solve(prob)


def launch(backend, cat, res, ctx=None):
    import kpamd
    from kpamd import catalog as cmod
    reqs = kpamd.launch_requests_from_solve(res)
    if backend == "device":
        ch = kpamd.Catalog(ctx, cat)
        plan = kpamd.LaunchPlan(ctx, ch, reqs, cmod.ZONES)
        try:
            out, _ = plan.run(read=True)
        finally:
            plan.close()
            ch.close()
        return out
    from oracle import pyoracle
    return pyoracle.launch_select(cat, reqs, cmod.ZONES)


def launched_reservation(cat, nc, lr):
    """The reservation a reserved launch goes into: the override's (type, zone) reserved offering compatible with the
    NodeClaim's reservation-id requirement, of the launch's reservation type, with the greatest capacity (the
    ReservedOfferingFilter's per-zone choice, R:pkg/providers/instance/filter/filter.go:222-274)."""
    assert lr["capacity_type"] == "reserved"
    t, z = lr["overrides"][0]
    ids = next((r[2] for r in nc["requirements"] if r[0] == RID), None)
    offs = [o for o in cat[t].offerings if o.capacity_type == "reserved" and o.zone == z and o.available
            and o.reservation_type == lr["reservation_type"] and (ids is None or o.reservation_id in ids)]
    return max(offs, key=lambda o: o.reservation_capacity).reservation_id


def req_of(nc, key):
    return next((r for r in nc["requirements"] if r[0] == key), None)


BACKENDS = ["oracle", pytest.param("device", marks=pytest.mark.gpu)]


def _be(request, backend):
    return (backend, request.getfixturevalue("ctx")) if backend == "device" else (backend, None)


@pytest.mark.parametrize("backend", BACKENDS)
def test_mark_capacity_reservations_as_launched(request, backend, lib):
    """R:pkg/cloudprovider/suite_test.go:1453-1461: a pod on the reserved-only NodePool gets one NodeClaim; launching it
    takes one instance of the reservation (10 -> 9)."""
    from kpamd.model import PodShape
    be, ctx = _be(request, backend)
    cat = suite_catalogue(lib)
    res = solve(be, problem(cat, [reserved_pool()], [PodShape({})], [1], STRICT), ctx)
    assert len(res["nodeclaims"]) == 1 and res["placement"][0] == 0
    nc = res["nodeclaims"][0]
    assert req_of(nc, RID)[:3] == (RID, "In", sorted(f"cr-m5.large-1a-{rt}" for rt in RTYPES))
    lr = launch(be, cat, res, ctx)[0]
    assert lr["status"] == 0 and lr["capacity_type"] == "reserved"
    counts = {f"cr-m5.large-1a-{rt}": 10 for rt in RTYPES}
    counts[launched_reservation(cat, nc, lr)] -= 1  # CapacityReservationProvider.MarkLaunched
    assert sorted(counts.values()) == [9, 10]
    assert counts["cr-m5.large-1a-default"] == 9  # CapacityReservationTypeFilter: default before capacity-block


@pytest.mark.parametrize("backend", BACKENDS)
@pytest.mark.parametrize("crt", RTYPES)
def test_capacity_reservation_labels(request, backend, lib, crt):
    """R:pkg/cloudprovider/suite_test.go:1482-1505: a pod selecting a reservation type lands on a NodeClaim launched
    into that type's reservation, labelled reserved / its id / its type."""
    from kpamd.model import PodShape
    be, ctx = _be(request, backend)
    cat = suite_catalogue(lib)
    res = solve(be, problem(cat, [reserved_pool()], [PodShape({}, node_selector={RT: crt})], [1], STRICT), ctx)
    assert len(res["nodeclaims"]) == 1
    nc = res["nodeclaims"][0]
    assert req_of(nc, RID)[:3] == (RID, "In", [f"cr-m5.large-1a-{crt}"])
    assert req_of(nc, RT)[:3] == (RT, "In", [crt])
    lr = launch(be, cat, res, ctx)[0]
    assert lr["capacity_type"] == "reserved" and lr["reservation_type"] == crt
    assert launched_reservation(cat, nc, lr) == f"cr-m5.large-1a-{crt}"


def _big_pods_problem(lib, mode, cap=2, n=5):
    """Reserved-only NodePool over m5.large / c5.large, one m5.large reservation of `cap`; every pod fills a node."""
    from kpamd import catalog as cmod
    from kpamd.model import PodShape
    crs = [cmod.CapacityReservation("cr-a", "m5.large", "test-zone-1a", "default", cap)]
    cat = cmod.build_catalog(lib, rows=_rows(["c5.large", "m5.large"]), capacity_reservations=crs)
    return cat, problem(cat, [reserved_pool()], [PodShape({"cpu": 1500})], [n], mode)


@pytest.mark.parametrize("backend", BACKENDS)
def test_strict_stops_at_reservation_capacity(request, backend, lib):
    """Strict mode: the third NodeClaim cannot reserve (capacity 2 spent) and the reserved-only pool has nothing else:
    the pods wait (ReservedOfferingError, not relaxed)."""
    be, ctx = _be(request, backend)
    cat, prob = _big_pods_problem(lib, STRICT)
    res = solve(be, prob, ctx)
    assert len(res["nodeclaims"]) == 2
    assert (res["placement"] >= 0).sum() == 2
    assert all(req_of(n, RID)[:3] == (RID, "In", ["cr-a"]) for n in res["nodeclaims"])
    assert res["stats"]["reserved_offering_errors"] >= 3


@pytest.mark.parametrize("backend", BACKENDS)
def test_fallback_keeps_scheduling_without_reservations(request, backend, lib):
    """Fallback mode (the scheduler default): an Add never fails for want of capacity; the NodeClaims past the cap hold
    no reservation and carry no reservation-id requirement."""
    be, ctx = _be(request, backend)
    cat, prob = _big_pods_problem(lib, FALLBACK)
    res = solve(be, prob, ctx)
    assert len(res["nodeclaims"]) == 5 and (res["placement"] >= 0).all()
    held = [req_of(n, RID) for n in res["nodeclaims"]]
    assert [h is not None and h[1] == "In" for h in held] == [True, True, False, False, False]
    assert res["stats"]["reserved_offering_errors"] == 0


@pytest.mark.parametrize("backend", BACKENDS)
def test_release_when_nodeclaim_narrows(request, backend, lib):
    """A NodeClaim holding the only m5.large reservation narrows to m5.xlarge when a pod pinned to it joins: the
    reservation goes back, and a later pod pinned to m5.large reserves it on a new NodeClaim (strict mode)."""
    from kpamd import catalog as cmod
    from kpamd.model import NodePool, PodShape
    be, ctx = _be(request, backend)
    crs = [cmod.CapacityReservation("cr-a", "m5.large", "test-zone-1a", "default", 1)]
    cat = cmod.build_catalog(lib, rows=_rows(["m5.large", "m5.xlarge"]), capacity_reservations=crs)
    pool = NodePool("default", 0, 0, [(CT, "In", ["reserved", "on-demand"]), (ZONE, "In", ["test-zone-1a"])])
    shapes = [PodShape({"cpu": 300}), PodShape({"cpu": 200}, node_selector={IT: "m5.xlarge"}),
              PodShape({"cpu": 1700}, node_selector={IT: "m5.large"})]
    res = solve(be, problem(cat, [pool], shapes, [1, 1, 1], STRICT), ctx)
    assert (res["placement"] >= 0).all()
    ncs = res["nodeclaims"]
    assert len(ncs) == 2
    by_pod = {p: i for i, n in enumerate(ncs) for p in n["pods"]}
    large = ncs[by_pod[2]]
    assert req_of(large, RID)[:3] == (RID, "In", ["cr-a"])
    xl = ncs[by_pod[1]]
    assert by_pod[0] == by_pod[1] and req_of(xl, RID) is None


# ---- device == oracle on randomized batches ----------------------------------------------------------------------
def random_reserved_problem(cat, n_pods, seed, mode):
    from kpamd import synth
    from kpamd.model import NodePool
    prob = synth.config2(cat, n_pods=n_pods, seed=seed, n_shapes=48)
    rng = np.random.default_rng(seed + 100)
    for i, sh in enumerate(prob.shapes):
        if i % 7 == 3:
            sh.node_selector = dict(sh.node_selector, **{RT: str(rng.choice(RTYPES))})
        elif i % 11 == 5:
            sh.required_terms = [[(CT, "In", ["reserved"])]]
    prob.nodepools = [NodePool("reserved-first", 20, 0, [(CT, "In", ["reserved"])]),
                      NodePool("general", 10, 0, [(CT, "In", ["reserved", "on-demand", "spot"]),
                                                  (K + "instance-generation", "Gt", ["2"])])] + prob.nodepools[1:]
    prob.reserved_offering_mode = mode
    return prob


@pytest.mark.parametrize("seed,mode", [(0, STRICT), (1, FALLBACK), (2, STRICT), (3, FALLBACK)])
def test_oracle_random_reserved_runs(catalog, seed, mode):
    from oracle import pyoracle
    from test_reserved_offerings import reserved_catalogue
    cat = reserved_catalogue(catalog, 300, seed)
    res = pyoracle.solve(random_reserved_problem(cat, 800, seed, mode))
    held = sum(req_of(n, RID) is not None for n in res["nodeclaims"])
    assert held > 0
    if mode == STRICT:
        assert res["stats"]["reserved_offering_errors"] >= 0


@pytest.mark.gpu
@pytest.mark.parametrize("seed,mode", [(0, STRICT), (1, FALLBACK), (2, STRICT), (3, FALLBACK), (4, STRICT)])
def test_device_random_reserved_matches_oracle(ctx, catalog, seed, mode):
    import kpamd
    from oracle import pyoracle
    from test_gpu_parity import check_same
    from test_reserved_offerings import reserved_catalogue
    cat = reserved_catalogue(catalog, 300 if seed % 2 else len(catalog), seed)
    prob = random_reserved_problem(cat, 2500, seed, mode)
    got = kpamd.Scheduler(ctx, prob).solve()
    want = pyoracle.solve(prob)
    check_same(got, want)
    assert got["stats"]["reserved_offering_errors"] == want["stats"]["reserved_offering_errors"]
    assert sum(req_of(n, RID) is not None for n in got["nodeclaims"]) > 0


@pytest.mark.gpu
def test_device_reserved_solve_refresh_matches_oracle(ctx, catalog):
    """A strict-mode Solve plan on a reservation catalogue, refreshed in place after reservation capacity / ICE
    updates by id (kp_catalog_update_offerings + kp_solve_refresh: the capacities the ReservationManager starts from
    are recomputed), equals the oracle on the updated catalogue; and the refreshed plan differs from its first run."""
    import kpamd
    from oracle import pyoracle
    from test_gpu_parity import check_same
    from test_reserved_offerings import reserved_catalogue
    cat = reserved_catalogue(catalog, 300, 0)
    prob = random_reserved_problem(cat, 1500, 0, STRICT)
    sched = kpamd.Scheduler(ctx, prob)
    plan = sched.prepare()
    try:
        first = plan.run()
        ch = sched.catalogs[0]
        ups, k = [], 0
        for ti, t in enumerate(ch.instance_types):
            for o in t.offerings:
                if o.reservation_id:
                    cap = [0, 1, 2][k % 3]
                    k += 1
                    ups.append((ti, "reserved", o.zone, cap != 0, None, o.reservation_id, cap))
        assert ups
        ch.update_offerings(ups, ch.seqnum() + 1)
        plan.refresh()
        got = plan.run()
    finally:
        plan.close()
        for c in sched.catalogs:
            c.close()
    want = pyoracle.solve(prob)  # prob's catalogue objects carry the updates
    check_same(got, want)
    assert got["stats"]["reserved_offering_errors"] == want["stats"]["reserved_offering_errors"]
    assert ([n["requirements"] for n in got["nodeclaims"]] != [n["requirements"] for n in first["nodeclaims"]]
            or got["stats"]["reserved_offering_errors"] != first["stats"]["reserved_offering_errors"])
