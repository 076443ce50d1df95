"""Consolidation over capacity-reservation catalogues (ABI v10): SimulateScheduling builds its scheduler with
DisableReservedCapacityFallback, so every simulation reserves offerings strictly; a reserved offering is
priced on-demand / 1e7 (R:pkg/providers/instancetype/offering/offering.go:160-166), and a candidate node launched into
a reservation is priced by its reservation's offering (getCandidatePrices: the offerings compatible with the node's
labels, reservation id included).

Written-spec KATs from the design R:designs/odcr.md:341-369 ("Consolidating into Capacity Reserved Instances": an
on-demand node whose pods fit a reserved type is replaced into the reservation; "Consolidating between Capacity
Reservations": a node in a large reservation moves to a small one when its pods scale down), plus the strict cap
(an exhausted reservation is not used: the replacement is on-demand). Each KAT runs on the oracle (CPU) and on the
device (-m gpu, which must also equal the oracle); randomized reservation clusters check device == oracle. Upstream
SimulateScheduling is not in the container: parity unpinned beyond the design's written behaviour.
"""
import numpy as np
import pytest

from kpamd import catalog as cmod

ZONE_A = "test-zone-1a"
RID = "karpenter.k8s.aws/capacity-reservation-id"
RTYPE = "karpenter.k8s.aws/capacity-reservation-type"
REPLACE, DELETE, NOOP = 2, 1, 0


def _catalogue(lib, names, reservations):
    table = {r["name"]: r for r in cmod.load_ec2_table()}
    return cmod.build_catalog(lib, rows=[table[n] for n in names], capacity_reservations=reservations)


def _od(cat, name):
    it = next(t for t in cat if t.name == name)
    return min(o.price for o in it.offerings if o.capacity_type == "on-demand" and o.zone == ZONE_A)


def _cluster(cat, node_type, capacity_type, pods, reservation=None, pool_cts=("on-demand", "spot", "reserved")):
    """One node of node_type in test-zone-1a (launched into `reservation` when given) running `pods` pods of 500m /
    1Gi, and one NodePool admitting the capacity types pool_cts."""
    from kpamd import synth
    from kpamd.model import Cluster, ClusterNode, ExistingNode, NodePool, PodShape
    ti = next(i for i, t in enumerate(cat) if t.name == node_type)
    it = cat[ti]
    labels = synth.node_labels(it, 0, capacity_type, "default", "node-00000")
    if reservation:
        labels[RID], labels[RTYPE] = reservation.id, reservation.reservation_type
    shape = PodShape(synth.req_res(500, 1024))
    alloc = it.allocatable()
    used = {"cpu": 500 * pods, "memory": 1024 * synth.MI * 1000 * pods, "pods": 1000 * pods}
    node = ClusterNode(ExistingNode("node-00000", labels, {r: alloc[r] - used[r] for r in used}, {}, [], True), 0, ti,
                       list(range(pods)))
    pool = NodePool("default", 0, 0, [("karpenter.sh/capacity-type", "In", list(pool_cts))])
    return Cluster([cat], [pool], [node], [shape], np.zeros(pods, np.uint32),
                   (1_750_000_000 + np.arange(pods)).astype(np.int64), np.arange(1, pods + 1, dtype=np.uint64),
                   candidates=[0], name="reserved-cluster")


def _simulate(request, backend, cl):
    if backend == "oracle":
        from oracle import pyoracle
        return pyoracle.simulate_batch(cl, [[0]], multi_node=False)[0][0]
    import kpamd
    from oracle import pyoracle
    ctx = request.getfixturevalue("ctx")
    plan = kpamd.ClusterPlan(ctx, cl)
    try:
        got = plan.simulate([[0]], multi_node=False)[0][0]
    finally:
        plan.close()
    want = pyoracle.simulate_batch(cl, [[0]], multi_node=False)[0][0]
    assert {k: got[k] for k in want} == want, (got, want)
    return got


BACKENDS = ["oracle", pytest.param("device", marks=pytest.mark.gpu)]


@pytest.mark.parametrize("backend", BACKENDS)
def test_consolidate_into_a_reservation(request, lib, backend):
    """odcr.md:341-346: an on-demand m5.xlarge whose two pods fit an m5.large with an available reservation is replaced
    into the reservation (its price on-demand / 1e7)."""
    cr = cmod.CapacityReservation("cr-m5.large-1a", "m5.large", ZONE_A, "default", 1)
    cat = _catalogue(lib, ["m5.large", "m5.xlarge", "m5.2xlarge"], [cr])
    r = _simulate(request, backend, _cluster(cat, "m5.xlarge", "on-demand", 2))
    assert r["decision"] == REPLACE
    assert r["replacement_price"] == pytest.approx(_od(cat, "m5.large") / 1e7)
    assert r["candidate_price"] == pytest.approx(_od(cat, "m5.xlarge"))


@pytest.mark.parametrize("backend", BACKENDS)
def test_consolidate_between_reservations(request, lib, backend):
    """odcr.md:353-369: a c6a.48xlarge launched into a reservation (priced c6a.48xlarge on-demand / 1e7) holding one
    small pod moves into a c6a.large reservation, whose near-0 price is lower still."""
    big = cmod.CapacityReservation("cr-c6a.48xlarge-1a", "c6a.48xlarge", ZONE_A, "default", 0)  # in use by the node
    small = cmod.CapacityReservation("cr-c6a.large-1a", "c6a.large", ZONE_A, "default", 1)
    cat = _catalogue(lib, ["c6a.large", "c6a.xlarge", "c6a.48xlarge"], [big, small])
    r = _simulate(request, backend, _cluster(cat, "c6a.48xlarge", "reserved", 1, reservation=big))
    assert r["candidate_price"] == pytest.approx(_od(cat, "c6a.48xlarge") / 1e7)
    assert r["decision"] == REPLACE
    assert r["replacement_price"] == pytest.approx(_od(cat, "c6a.large") / 1e7)


@pytest.mark.parametrize("backend", BACKENDS)
def test_exhausted_reservation_is_not_used(request, lib, backend):
    """Strict reservations: with no capacity left the reserved offering is unavailable; the replacement (a NodePool of
    on-demand and reserved capacity) is the cheaper on-demand m5.large."""
    cr = cmod.CapacityReservation("cr-m5.large-1a", "m5.large", ZONE_A, "default", 0)
    cat = _catalogue(lib, ["m5.large", "m5.xlarge", "m5.2xlarge"], [cr])
    r = _simulate(request, backend, _cluster(cat, "m5.xlarge", "on-demand", 2, pool_cts=("on-demand", "reserved")))
    assert r["decision"] == REPLACE
    assert r["replacement_price"] == pytest.approx(_od(cat, "m5.large"))


def reservation_cluster(catalog, seed, n_nodes=8):
    """A random cluster whose catalogue holds reservations for a few of its types (capacities 0-3) and some of whose
    nodes were launched into them."""
    from kpamd import synth
    cl = synth.random_cluster(catalog, seed, n_nodes=n_nodes)
    rng = np.random.default_rng(seed)
    names = sorted({cl.catalogs[0][n.instance_type].name for n in cl.nodes})
    picks = list(rng.choice(names, size=min(4, len(names)), replace=False))
    crs = [cmod.CapacityReservation(f"cr-{n}-{z}", str(n), z, str(rng.choice(["default", "capacity-block"])),
                                    int(rng.integers(0, 4))) for n in picks for z in cmod.ZONES[:2]]
    return cl, crs


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [70, 72, 74, 76, 78, 79])
def test_gpu_random_reservation_clusters(ctx, lib, catalog, seed, general_mode):
    from test_gpu_consolidation import check
    from kpamd import synth
    cl, crs = reservation_cluster(catalog, seed)
    cl = _reserve_nodes(lib, cl, crs, launch_into=seed % 2 == 0)
    subs = synth.consolidation_subsets(cl, 12, seed=seed, max_size=4) + [[c] for c in cl.candidates[:8]]
    check(ctx, cl, subs, multi_node=bool(seed % 3))


def _reserve_nodes(lib, cl, crs, launch_into):
    """cl's catalogue rebuilt with the reservations; with launch_into, the nodes of a reserved type in its zone carry
    the reservation's labels (launched into it)."""
    table = {r["name"]: r for r in cmod.load_ec2_table()}
    cat = cmod.build_catalog(lib, rows=[table[it.name] for it in cl.catalogs[0]], capacity_reservations=crs)
    by = {cr.instance_type: cr for cr in crs}
    for n in cl.nodes:
        cr = by.get(cat[n.instance_type].name)
        if launch_into and cr and n.node.labels.get("topology.kubernetes.io/zone") == cr.availability_zone:
            n.node.labels = dict(n.node.labels, **{"karpenter.sh/capacity-type": "reserved", RID: cr.id,
                                                  RTYPE: cr.reservation_type})
    for p in cl.nodepools:  # every capacity type admitted: reserved offerings are reachable
        p.requirements = [r for r in p.requirements if r[0] != "karpenter.sh/capacity-type"]
    cl.catalogs = [cat]
    return cl


@pytest.mark.parametrize("seed", [70, 76])
def test_oracle_random_reservation_clusters(lib, catalog, seed):
    from kpamd import synth
    from oracle import pyoracle
    cl, crs = reservation_cluster(catalog, seed)
    cl = _reserve_nodes(lib, cl, crs, launch_into=seed % 2 == 0)
    assert any(n.node.labels.get("karpenter.sh/capacity-type") == "reserved" for n in cl.nodes)
    subs = synth.consolidation_subsets(cl, 12, seed=seed, max_size=4) + [[c] for c in cl.candidates[:8]]
    res, _ = pyoracle.simulate_batch(cl, subs)
    assert {DELETE, REPLACE} <= {r["decision"] for r in res}
