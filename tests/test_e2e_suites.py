"""The reference's e2e expectations for scheduling and consolidation (R:test/suites/scheduling/suite_test.go,
R:test/suites/consolidation/suite_test.go), transcribed over the cluster model of tests/e2e.py: provision, scale,
consolidate to a fixed point, then assert what each suite asserts. Every scenario runs on the oracle (CPU) and on the
device (-m gpu); on the device the whole trajectory (every node launched, every command) must also equal the oracle's.

These are the only reference-held statements of consolidation outcomes; upstream core (sigs.k8s.io/karpenter) is not in
the container, so the disruption-cost tie order, the ReplicaSet victim order and CreateFleet's allocation are the
model's (tests/e2e.py docstring), and the assertions are the suites' own, not exact node lists.
"""
import pytest

import e2e
from e2e import CT, IT, K, NOT_BURSTABLE, RID, RTYPE, ZONE, ZONE_ID

BACKENDS = ["oracle", pytest.param("device", marks=pytest.mark.gpu)]
SIZE = K + "instance-size"


@pytest.fixture
def mk(request, lib):
    envs = []

    def make(backend, **kw):
        ctx = request.getfixturevalue("ctx") if backend == "device" else None
        env = e2e.Env(backend, lib, ctx=ctx, **kw)
        envs.append(env)
        return env
    yield make
    for env in envs:
        env.close()


def _twin(mk, backend, scenario):
    """Run scenario(env) on the backend; on the device also on the oracle, and require the same trajectory."""
    env = mk(backend)
    out = scenario(env)
    if backend == "device":
        ref = mk("oracle")
        want = scenario(ref)
        assert env.launches == ref.launches, (env.launches, ref.launches)
        assert [(c.method, c.candidates, c.decision) for c in env.commands] == \
            [(c.method, c.candidates, c.decision) for c in ref.commands]
        assert env.summary() == ref.summary()
        assert out == want
    return env


def _pod(cpu_m=0, **kw):
    from kpamd.model import PodShape
    req = {"pods": 1000}
    if cpu_m:
        req["cpu"] = cpu_m
    return PodShape(req, **kw)


def _spread(key, app, min_domains=None):
    from kpamd.model import LabelSelector, TopologySpread
    return TopologySpread(key, 1, LabelSelector({"app": app}), "DoNotSchedule", min_domains)


# ---- R:test/suites/consolidation/suite_test.go ---------------------------------------------------------------------
@pytest.mark.parametrize("backend", BACKENDS)
@pytest.mark.parametrize("capacity_type", ["on-demand", "spot"])
@pytest.mark.parametrize("scale_down", ["ranked", 1, 3])
def test_consolidation_delete(mk, backend, capacity_type, scale_down):
    """:487-569 "should consolidate nodes (delete)": 100 one-CPU pods on medium/large/xlarge nodes (no burstable
    families); the Deployment scales to 40 and average CPU utilization drops below 0.5; consolidation then raises it
    above 0.6. Both capacity types. The ReplicaSet's own victim order empties whole nodes (Emptiness alone then
    suffices); a random scale-down (seeded) leaves partly used nodes, which multi-node consolidation has to pack."""
    from kpamd.model import NodePool

    def scenario(env):
        env.pools = [NodePool("default", 0, 0, [(CT, "In", [capacity_type]), (SIZE, "In", ["medium", "large", "xlarge"]),
                                                NOT_BURSTABLE])]
        env.deploy("large-app", _pod(1000, labels={"app": "large-app"}), 100)
        env.provision()
        assert not env.pending()
        env.scale("large-app", 40, seed=None if scale_down == "ranked" else scale_down)
        low = env.utilization()
        assert low < 0.5, low
        cmds = env.consolidate()
        if scale_down != "ranked":
            assert any(c.method != "emptiness" for c in cmds), cmds
        high = env.utilization()
        assert high > 0.6, high
        assert not env.pending()
        assert all(v["ct"] == capacity_type for v in env.nodes.values())
        return round(low, 6), round(high, 6), len(env.nodes)
    _twin(mk, backend, scenario)


@pytest.mark.parametrize("backend", BACKENDS)
@pytest.mark.parametrize("capacity_type", ["on-demand", "spot"])
def test_consolidation_replace(mk, backend, capacity_type):
    """:570-725 "should consolidate nodes (replace)": three 4-CPU and three 1.8-CPU pods, each Deployment spread over
    hostnames (maxSkew 1), on large/2xlarge linux nodes: three nodes. The 4-CPU Deployment scales to 0 (utilization
    < 0.5); consolidation replaces each node in turn (the spread keeps the small pods apart) by a .large: utilization
    > 0.8, exactly three .large nodes and no other. Spot nodes are replaced spot-to-spot."""
    from kpamd.model import NodePool

    def scenario(env):
        env.pools = [NodePool("default", 0, 0, [(CT, "In", [capacity_type]), (SIZE, "In", ["large", "2xlarge"]),
                                                NOT_BURSTABLE, ("kubernetes.io/os", "In", ["linux"])])]
        env.deploy("large-app", _pod(4000, labels={"app": "large-app"},
                                     topology_spread=[_spread("kubernetes.io/hostname", "large-app")]), 3)
        env.deploy("small-app", _pod(1800, labels={"app": "small-app"},
                                     topology_spread=[_spread("kubernetes.io/hostname", "small-app")]), 3)
        env.provision()
        assert not env.pending()
        assert len(env.nodes) == 3, env.summary()  # "3 nodes due to the anti-affinity rules"
        env.scale("large-app", 0)
        assert env.utilization() < 0.5
        cmds = env.consolidate()
        assert env.utilization() > 0.8, env.summary()
        names = [env.type_of(n) for n in env.nodes]
        assert sum(n.endswith(".large") for n in names) == 3, names
        assert len(names) == 3, names
        assert all(v["ct"] == capacity_type for v in env.nodes.values())
        assert all(c.method == "single" and c.decision == 2 for c in cmds), cmds
        return names
    _twin(mk, backend, scenario)


@pytest.mark.parametrize("backend", BACKENDS)
def test_consolidation_on_demand_to_spot(mk, backend):
    """:726-850 "should consolidate on-demand nodes to spot (replace)": two 1.8-CPU pods spread over hostnames on
    on-demand .large nodes; the NodePool then admits every capacity type (capacity-type Exists) and consolidation
    replaces both nodes with spot nodes, leaving no other node."""
    from kpamd.model import NodePool

    def scenario(env):
        env.pools = [NodePool("default", 0, 0, [(CT, "In", ["on-demand"]), (SIZE, "In", ["large"]), NOT_BURSTABLE])]
        env.deploy("small-app", _pod(1800, labels={"app": "small-app"},
                                     topology_spread=[_spread("kubernetes.io/hostname", "small-app")]), 2)
        env.provision()
        assert len(env.nodes) == 2 and all(v["ct"] == "on-demand" for v in env.nodes.values())
        # coretest.ReplaceRequirements: the keys given replace theirs, the others stay
        env.pools[0].requirements = [(CT, "Exists", []), (SIZE, "In", ["large"]), NOT_BURSTABLE]
        env.consolidate()
        cts = [v["ct"] for v in env.nodes.values()]
        assert cts == ["spot", "spot"], env.summary()
        return env.summary()
    _twin(mk, backend, scenario)


def _reservation(cid, it, count):
    from kpamd import catalog as cmod
    return cmod.CapacityReservation(cid, it, "test-zone-1a", "default", count)


@pytest.mark.parametrize("backend", BACKENDS)
def test_consolidation_into_a_reservation(mk, backend):
    """:911-957 "should consolidate into a reserved offering": a pod restricted to m5.large / m5.xlarge lands on an
    on-demand m5.large; once the EC2NodeClass selects an m5.xlarge reservation, the node is replaced by a reserved
    m5.xlarge in that reservation ("already paid for")."""
    from kpamd.model import NodePool

    def scenario(env):
        env.pools = [NodePool("default", 0, 0, [(CT, "In", ["on-demand", "reserved"])])]
        env.deploy("app", _pod(required_terms=[[(IT, "In", ["m5.large", "m5.xlarge"])]]), 1)
        env.provision()
        (n0, v0), = env.nodes.items()
        assert (env.type_of(n0), v0["ct"]) == ("m5.large", "on-demand")
        env.add_reservation(_reservation("cr-xlarge", "m5.xlarge", 1))
        env.consolidate()
        (n1, v1), = env.nodes.items()
        assert (env.type_of(n1), v1["ct"], v1["rid"]) == ("m5.xlarge", "reserved", "cr-xlarge")
        assert env.labels(n1)[RID] == "cr-xlarge" and env.labels(n1)[CT] == "reserved"
        return env.summary()
    _twin(mk, backend, scenario)


@pytest.mark.parametrize("backend", BACKENDS)
def test_consolidation_between_reservations(mk, backend):
    """:958-1000 "should consolidate between reserved offerings": with only the m5.xlarge reservation selected the pod
    lands on a reserved m5.xlarge; adding an m5.large reservation consolidates it into a reserved m5.large."""
    from kpamd.model import NodePool

    def scenario(env):
        env.pools = [NodePool("default", 0, 0, [(CT, "In", ["on-demand", "reserved"])])]
        env.add_reservation(_reservation("cr-xlarge", "m5.xlarge", 1))
        env.deploy("app", _pod(required_terms=[[(IT, "In", ["m5.large", "m5.xlarge"])]]), 1)
        env.provision()
        (n0, v0), = env.nodes.items()
        assert (env.type_of(n0), v0["ct"], v0["rid"]) == ("m5.xlarge", "reserved", "cr-xlarge")
        env.add_reservation(_reservation("cr-large", "m5.large", 1))
        env.consolidate()
        (n1, v1), = env.nodes.items()
        assert (env.type_of(n1), v1["ct"], v1["rid"]) == ("m5.large", "reserved", "cr-large")
        return env.summary()
    _twin(mk, backend, scenario)


# ---- R:test/suites/scheduling/suite_test.go --------------------------------------------------------------------------
@pytest.mark.parametrize("backend", BACKENDS)
def test_self_affinity_deployment(mk, backend):
    """:375-396 "should provision a node for a self-affinity deployment": two replicas with a required pod affinity to
    themselves on the hostname key share one node."""
    from kpamd.model import LabelSelector, PodAffinityTerm

    def scenario(env):
        env.pools = [e2e.default_nodepool()]
        env.deploy("self", _pod(labels={"test": "self-affinity"},
                                required_affinity=[PodAffinityTerm("kubernetes.io/hostname",
                                                                   LabelSelector({"test": "self-affinity"}))]), 2)
        env.provision()
        assert not env.pending() and len(env.nodes) == 1
        return env.summary()
    _twin(mk, backend, scenario)


@pytest.mark.parametrize("backend", BACKENDS)
def test_zonal_spread_min_domains(mk, backend):
    """:397-424 "should provision three nodes for a zonal topology spread": three replicas spread over zones (maxSkew 1,
    minDomains 3) get three nodes, one per zone."""
    def scenario(env):
        env.pools = [e2e.default_nodepool()]
        env.deploy("zonal", _pod(labels={"app": "zonal-spread"}, topology_spread=[_spread(ZONE, "zonal-spread", 3)]), 3)
        env.provision()
        assert not env.pending() and len(env.nodes) == 3
        assert sorted(v["zone"] for v in env.nodes.values()) == ["test-zone-1a", "test-zone-1b", "test-zone-1c"]
        return env.summary()
    _twin(mk, backend, scenario)


@pytest.mark.parametrize("backend", BACKENDS)
def test_higher_priority_nodepool(mk, backend):
    """:425-493 "should provision a node using a NodePool with higher priority": weight 10 (t3.nano) and weight 100
    (c5.large) pools: one node, a c5.large from the weight-100 pool."""
    from kpamd.model import NodePool

    def scenario(env):
        env.pools = [NodePool("low", 10, 0, [("kubernetes.io/os", "In", ["linux"]), (IT, "In", ["t3.nano"])]),
                     NodePool("high", 100, 0, [("kubernetes.io/os", "In", ["linux"]), (IT, "In", ["c5.large"])])]
        env.deploy("pod", _pod(), 1)
        env.provision()
        (n, v), = env.nodes.items()
        assert env.type_of(n) == "c5.large" and env.pools[v["pool"]].name == "high"
        return env.summary()
    _twin(mk, backend, scenario)


@pytest.mark.parametrize("backend", BACKENDS)
def test_overlapping_zone_and_zone_id(mk, backend):
    """:631-657 "should provision a node for a pod with overlapping zone and zone-id requirements": zone In {z0, z1} and
    zone-id In {id1, id2} meet only in z1: the node is in z1 with z1's zone id."""
    def scenario(env):
        env.pools = [e2e.default_nodepool()]
        env.deploy("pod", _pod(required_terms=[[(ZONE, "In", ["test-zone-1a", "test-zone-1b"]),
                                                (ZONE_ID, "In", ["tstz1-1b", "tstz1-1c"])]]), 1)
        env.provision()
        (n, v), = env.nodes.items()
        assert env.labels(n)[ZONE] == "test-zone-1b" and env.labels(n)[ZONE_ID] == "tstz1-1b"
        return env.summary()
    _twin(mk, backend, scenario)


@pytest.mark.parametrize("backend", BACKENDS)
def test_zone_id_requirements_pick_their_zone(mk, backend):
    """:658-708 "should provision nodes for pods with zone-id requirements in the correct zone": the NodePool requires
    a custom label to exist; each pod names one zone through that label and its zone id: one node per zone, each in the
    zone its label names, with the matching zone id."""
    def scenario(env):
        from kpamd import catalog as cmod
        pool = e2e.default_nodepool()
        pool.requirements = [("expected-zone-label", "Exists", [])]  # coretest.ReplaceRequirements: only this key is new
        pool.requirements = e2e.default_nodepool().requirements + pool.requirements
        env.pools = [pool]
        for z, zid in zip(cmod.ZONES, cmod.ZONE_IDS):
            env.deploy(f"pod-{z}", _pod(required_terms=[[("expected-zone-label", "In", [z]), (ZONE_ID, "In", [zid])]]), 1)
        env.provision()
        assert not env.pending() and len(env.nodes) == 3
        for name, _, _, _, reqs in env.launches:
            want = {k: v for k, op, v, *_ in reqs if op == "In"}["expected-zone-label"]
            assert [env.labels(name)[ZONE]] == want
            assert env.labels(name)[ZONE_ID] == cmod.ZONE_IDS[cmod.ZONES.index(want[0])]
        return env.summary()
    _twin(mk, backend, scenario)


def _reserved_env(env):
    from kpamd.model import NodePool
    env.add_reservation(_reservation("cr-large", "m5.large", 1))
    env.add_reservation(_reservation("cr-xlarge", "m5.xlarge", 2))
    env.pools = [NodePool("default", 0, 0, [(CT, "In", ["on-demand", "reserved"]), ("kubernetes.io/os", "In", ["linux"])])]


@pytest.mark.parametrize("backend", BACKENDS)
def test_schedule_against_a_reservation_id(mk, backend):
    """:763-788 "should schedule against a specific reservation ID": the NodeClaim carries capacity-reservation-id In
    {the xlarge reservation}; the node is reserved, of reservation type default, in that reservation."""
    def scenario(env):
        _reserved_env(env)
        env.deploy("pod", _pod(required_terms=[[(RID, "In", ["cr-xlarge"])]]), 1)
        env.provision()
        (name, _, _, _, reqs), = env.launches
        assert {k: v for k, op, v, *_ in reqs if op == "In"}[RID] == ["cr-xlarge"]
        lab = env.labels(name)
        assert (lab[CT], lab[RTYPE], lab[RID]) == ("reserved", "default", "cr-xlarge")
        return env.summary()
    _twin(mk, backend, scenario)


@pytest.mark.parametrize("backend", BACKENDS)
def test_schedule_against_a_reservation_type(mk, backend):
    """:789-822 "should schedule against a specific reservation type": reservation type In {default} and instance type
    m5.xlarge: the NodeClaim carries the type requirement, the node is the xlarge reservation's."""
    def scenario(env):
        _reserved_env(env)
        env.deploy("pod", _pod(required_terms=[[(RTYPE, "In", ["default"]), (IT, "In", ["m5.xlarge"])]]), 1)
        env.provision()
        (name, _, _, _, reqs), = env.launches
        assert {k: v for k, op, v, *_ in reqs if op == "In"}[RTYPE] == ["default"]
        lab = env.labels(name)
        assert (lab[CT], lab[RTYPE], lab[RID]) == ("reserved", "default", "cr-xlarge")
        return env.summary()
    _twin(mk, backend, scenario)


@pytest.mark.parametrize("backend", BACKENDS)
def test_fall_back_when_reservations_are_exhausted(mk, backend):
    """:823-860 "should fall back when compatible capacity reservations are exhausted": two m5.large pods with hostname
    anti-affinity and one m5.large reservation: two NodeClaims, exactly one carrying capacity-reservation-id In {the
    large reservation}; two nodes."""
    from kpamd.model import LabelSelector, PodAffinityTerm

    def scenario(env):
        _reserved_env(env)
        env.deploy("pods", _pod(labels={"foo": "bar"}, required_terms=[[(IT, "In", ["m5.large"])]],
                                required_anti_affinity=[PodAffinityTerm("kubernetes.io/hostname",
                                                                        LabelSelector({"foo": "bar"}))]), 2)
        env.provision()
        assert not env.pending() and len(env.nodes) == 2
        rids = [{k: v for k, op, v, *_ in reqs if op == "In"}.get(RID) for _, _, _, _, reqs in env.launches]
        assert len(rids) == 2 and sorted(map(str, rids)) == sorted(map(str, [["cr-large"], None])), rids
        return env.summary()
    _twin(mk, backend, scenario)
