"""The reference's behavioural Solve tests, transcribed as scenarios with the reference's expected outcomes asserted
(SURVEY §8c item 4). Each runs on the oracle (CPU) and on the device path (-m gpu): Solve, launch selection,
fake CreateFleet with InsufficientCapacityPools, ICE marks, re-Solve (tests/scenarios.py).

  minValues -> 2 NodeClaims           R:pkg/cloudprovider/suite_test.go:347-447 (In), :448-545 (Exists), :546-652
                                      (minValues on two keys)
  ICE fallback to another type        R:pkg/providers/instancetype/suite_test.go:1999-2031
  ICE fallback to another zone        R:pkg/providers/instancetype/suite_test.go:2032-2058 (and :2112-2138, Habana)
  ICE fallback to smaller instances   R:pkg/providers/instancetype/suite_test.go:2059-2092
  ICE cache expiry                    R:pkg/providers/instancetype/suite_test.go:2093-2111
  on-demand when spot is ICE'd        R:pkg/providers/instancetype/suite_test.go:2139-2174
  ICE'd type stays listed             R:pkg/providers/instancetype/suite_test.go:2175-2226 (no available offering left)
  Windows PrivateIPv4Address          R:pkg/providers/instancetype/suite_test.go:639-706 (launched on a type the VPC
                                      limits table advertises; not scheduled on one it does not)
  capacity type                       R:pkg/providers/instancetype/suite_test.go:2229-2244 (default on-demand; spot when
                                      flexible to both)
"""
import pytest

from kpamd.model import NodePool, PodShape

K = "karpenter.k8s.aws/"
ZONE = "topology.kubernetes.io/zone"
IT = "node.kubernetes.io/instance-type"
CT = "karpenter.sh/capacity-type"
OD_POOL = [(CT, "In", ["on-demand"])]  # the instancetype suite's default NodePool (R:suite_test.go:150-171)

BACKENDS = ["oracle", pytest.param("device", marks=pytest.mark.gpu)]


@pytest.fixture
def mk(request, lib):
    """Env factory for the parametrized backend (device envs need the session ctx)."""
    import scenarios
    envs = []

    def make(backend, types, ice=()):
        ctx = request.getfixturevalue("ctx") if backend == "device" else None
        e = scenarios.Env(backend, types, ctx=ctx, ice_pools=ice)
        envs.append(e)
        return e
    yield make
    for e in envs:
        e.close()


def rq(cpu_m=0, **extra):
    r = {"pods": 1000}
    if cpu_m:
        r["cpu"] = cpu_m
    r.update(extra)
    return r


def labels_of(types, name):
    it = next(t for t in types if t.name == name)
    return {k: v[0] for k, op, v, *_ in it.requirements if op == "In" and len(v) == 1}


# ---- R:pkg/cloudprovider/suite_test.go MinValues ---------------------------------------------------------------
MIN_NAMES = ["c5.large", "m5.large", "r5.large"]  # MakeUniqueInstancesAndFamilies: one type per family


@pytest.mark.parametrize("backend", BACKENDS)
@pytest.mark.parametrize("variant", ["in", "exists"])
def test_minvalues_forces_two_nodeclaims(backend, variant, mk, lib):
    """Two 0.9-CPU pods; a 1-vCPU type fits one, an 8-vCPU type fits both; NodePool instance-type minValues 2 keeps
    the second pod from joining the first NodeClaim (only one type would remain), so two NodeClaims launch, each
    CreateFleet carrying >= 2 instance types (R:pkg/cloudprovider/suite_test.go:347-545)."""
    import scenarios
    types = scenarios.uniform_instances(lib, MIN_NAMES[:2], [1, 8], [0.002, 0.003])
    names = [t.name for t in types]
    if variant == "in":
        reqs = [(CT, "In", ["spot"]), (IT, "In", names, 2)]
    else:
        reqs = [(IT, "Exists", [], 2), (IT, "In", names, 1)]
    env = mk(backend, types)
    nodes, pod_node = env.provision([NodePool("default", 0, 0, reqs)], [PodShape(rq(900))], [2])
    assert pod_node[0] is not None and pod_node[1] is not None, "ExpectScheduled(pod1), ExpectScheduled(pod2)"
    assert pod_node[0] != pod_node[1], "node1.Name != node2.Name"
    assert len(nodes) == 2, "CreateFleet called twice"
    for n in nodes:
        assert len({t for t, _ in n["overrides"]}) >= 2, "overrides carry >= minValues instance types"


@pytest.mark.parametrize("backend", BACKENDS)
def test_minvalues_on_two_keys(backend, mk, lib):
    """instance-type minValues 2 and instance-family minValues 3 over a 1/4/8-vCPU trio: two NodeClaims, each
    CreateFleet carrying exactly 3 types of 3 families (R:pkg/cloudprovider/suite_test.go:546-652)."""
    import scenarios
    types = scenarios.uniform_instances(lib, MIN_NAMES, [1, 4, 8], [0.002, 0.003, 0.004])
    names = [t.name for t in types]
    fams = [n.split(".")[0] for n in names]
    reqs = [(IT, "In", names, 2), (K + "instance-family", "In", fams, 3)]
    env = mk(backend, types)
    nodes, pod_node = env.provision([NodePool("default", 0, 0, reqs)], [PodShape(rq(900))], [2])
    assert None not in pod_node and pod_node[0] != pod_node[1]
    assert len(nodes) == 2
    for n in nodes:
        assert len({t for t, _ in n["overrides"]}) == 3
        assert len({t.split(".")[0] for t, _ in n["overrides"]}) == 3


# ---- R:pkg/providers/instancetype/suite_test.go: Insufficient Capacity Error Cache --------------------------------
@pytest.mark.parametrize("backend", BACKENDS)
def test_ice_fallback_to_other_type(backend, mk, lib):
    """inf2.24xlarge ICE'd on-demand in test-zone-1a: two 1-neuron pods first pack onto one inf2.24xlarge and stay
    pending; the second attempt launches two inferentia2 nodes (R:suite_test.go:1999-2031)."""
    import scenarios
    types = scenarios.fake_catalog(lib)
    env = mk(backend, types, ice=[("on-demand", "inf2.24xlarge", "test-zone-1a")])
    pool = [NodePool("default", 0, 0, OD_POOL)]
    shape = [PodShape(rq(**{"aws.amazon.com/neuron": 1000}), node_selector={ZONE: "test-zone-1a"})]
    nodes, pod_node = env.provision(pool, shape, [2])
    assert pod_node == [None, None], "ExpectNotScheduled: packed on one ICE'd inf2.24xlarge"
    nodes, pod_node = env.provision(pool, shape, [2])
    assert None not in pod_node and len({pod_node[0], pod_node[1]}) == 2, "two nodes"
    for n in nodes:
        assert labels_of(types, n["type"])[K + "instance-accelerator-name"] == "inferentia2"


@pytest.mark.parametrize("backend", BACKENDS)
@pytest.mark.parametrize("itype,res", [("p3.8xlarge", {"nvidia.com/gpu": 1000}), ("dl1.24xlarge", {"habana.ai/gaudi": 1000})])
def test_ice_fallback_to_other_zone(backend, itype, res, mk, lib):
    """The pod prefers test-zone-1a; the type's on-demand pool there is ICE'd: the first attempt fails, the second
    relaxes the preference and launches in test-zone-1b (R:suite_test.go:2032-2058, Habana :2112-2138)."""
    import scenarios
    types = scenarios.fake_catalog(lib)
    env = mk(backend, types, ice=[("on-demand", itype, "test-zone-1a")])
    pool = [NodePool("default", 0, 0, OD_POOL)]
    shape = [PodShape(rq(**res), node_selector={IT: itype}, preferred_terms=[(1, [(ZONE, "In", ["test-zone-1a"])])])]
    nodes, pod_node = env.provision(pool, shape, [1])
    assert pod_node == [None]
    nodes, pod_node = env.provision(pool, shape, [1])
    assert pod_node == [0]
    assert (nodes[0]["type"], nodes[0]["zone"]) == (itype, "test-zone-1b")


@pytest.mark.parametrize("backend", BACKENDS)
def test_ice_fallback_to_smaller_instances(backend, mk, lib):
    """m5.xlarge ICE'd in test-zone-1a; NodePool In {m5.large, m5.xlarge}; two 1-CPU pods pinned to test-zone-1a
    first pack onto an m5.xlarge (ICE), then launch as two m5.large (R:suite_test.go:2059-2092)."""
    import scenarios
    types = scenarios.fake_catalog(lib)
    env = mk(backend, types, ice=[("on-demand", "m5.xlarge", "test-zone-1a")])
    pool = [NodePool("default", 0, 0, OD_POOL + [("node.kubernetes.io/instance-type", "In", ["m5.large", "m5.xlarge"])])]
    shape = [PodShape(rq(1000), node_selector={ZONE: "test-zone-1a"})]
    nodes, pod_node = env.provision(pool, shape, [2])
    assert pod_node == [None, None]
    nodes, pod_node = env.provision(pool, shape, [2])
    assert None not in pod_node
    assert [n["type"] for n in nodes] == ["m5.large", "m5.large"]


@pytest.mark.parametrize("backend", BACKENDS)
def test_ice_cache_expiry(backend, mk, lib):
    """inf2.24xlarge (2 neuron) ICE'd: the pod stays pending; once the ICE entry is deleted (cache expiry) the
    next attempt launches inf2.24xlarge (R:suite_test.go:2093-2111)."""
    import scenarios
    types = scenarios.fake_catalog(lib)
    env = mk(backend, types, ice=[("on-demand", "inf2.24xlarge", "test-zone-1a")])
    pool = [NodePool("default", 0, 0, OD_POOL)]
    shape = [PodShape(rq(**{"aws.amazon.com/neuron": 2000}), node_selector={IT: "inf2.24xlarge"})]
    _, pod_node = env.provision(pool, shape, [1])
    assert pod_node == [None]
    env.ice.clear()  # InsufficientCapacityPools.Set([]) + UnavailableOfferingsCache.Delete(...)
    idx = [t.name for t in types].index("inf2.24xlarge")
    env.seq += 1
    if env.backend == "device":
        env.cat.update_offerings([(idx, "on-demand", "test-zone-1a", True)], seqnum=env.seq)
    else:
        for o in types[idx].offerings:
            if o.capacity_type == "on-demand" and o.zone == "test-zone-1a":
                o.available = True
    nodes, pod_node = env.provision(pool, shape, [1])
    assert pod_node == [0] and nodes[0]["type"] == "inf2.24xlarge"


@pytest.mark.parametrize("backend", BACKENDS)
def test_on_demand_when_spot_unavailable(backend, mk, lib):
    """Every type's spot pool in test-zone-1a is ICE'd; NodePool {spot, on-demand} x {test-zone-1a}: the first
    attempt launches spot and fails, the second falls back to on-demand (R:suite_test.go:2139-2174)."""
    import scenarios
    types = scenarios.fake_catalog(lib)
    env = mk(backend, types, ice=[("spot", t.name, "test-zone-1a") for t in types])
    pool = [NodePool("default", 0, 0, [(CT, "In", ["spot", "on-demand"]), (ZONE, "In", ["test-zone-1a"])])]
    shape = [PodShape(rq())]
    _, pod_node = env.provision(pool, shape, [1])
    assert pod_node == [None]
    nodes, pod_node = env.provision(pool, shape, [1])
    assert pod_node == [0] and nodes[0]["capacity_type"] == "on-demand"


@pytest.mark.parametrize("backend", BACKENDS)
def test_all_instance_types_listed_after_ice(backend, mk, lib):
    """m5.xlarge's on-demand and spot pools in test-zone-1a/1b ICE'd; four pods pinned to each (capacity type, zone)
    try it and stay pending; GetInstanceTypes still returns m5.xlarge, with no available offering
    (R:suite_test.go:2175-2226). Device backend: the resident catalogue after the four ICE marks answers
    CompatibleAvailableFilter with nothing for m5.xlarge."""
    import numpy as np
    import scenarios
    types = scenarios.fake_catalog(lib)
    pools = [(ct, "m5.xlarge", z) for ct in ("on-demand", "spot") for z in ("test-zone-1a", "test-zone-1b")]
    env = mk(backend, types, ice=pools)
    pool = [NodePool("default", 0, 0, [(IT, "In", ["m5.xlarge"]), (CT, "In", ["spot", "on-demand"])])]
    for ct in ("on-demand", "spot"):
        for z in ("test-zone-1a", "test-zone-1b"):
            _, pod_node = env.provision(pool, [PodShape(rq(1000), node_selector={CT: ct, ZONE: z})], [1])
            assert pod_node == [None]
    listed = env.cat.instance_types if backend == "device" else types
    names = [t.name for t in listed]
    assert "m5.xlarge" in names
    m5x = listed[names.index("m5.xlarge")]
    assert [o for o in m5x.offerings if o.available] == []
    if backend == "device":
        import kpamd
        kept, _, _ = kpamd.compatible_available_filter(env.ctx, env.cat, [([], {"cpu": 1000})])
        assert not kept[0][names.index("m5.xlarge")] and kept[0].sum() > 0


@pytest.mark.parametrize("backend", BACKENDS)
@pytest.mark.parametrize("cts,want", [(["on-demand"], "on-demand"), (["spot", "on-demand"], "spot")])
def test_capacity_type(backend, cts, want, mk, lib):
    """Default NodePool launches on-demand; one flexible to spot and on-demand launches spot
    (R:suite_test.go:2229-2244)."""
    import scenarios
    types = scenarios.fake_catalog(lib)
    env = mk(backend, types)
    nodes, pod_node = env.provision([NodePool("default", 0, 0, [(CT, "In", cts)])], [PodShape(rq())], [1])
    assert pod_node == [0] and nodes[0]["capacity_type"] == want


PIP = "vpc.amazonaws.com/PrivateIPv4Address"


def _test_type_row():
    """The reference's fabricated "test" type (R:suite_test.go:657-680): 2 vCPU, 8 GiB, x86_64, 3 ENIs x 10 IPv4, absent
    from the VPC limits table (so PrivateIPv4Address capacity 0), offered in test-zone-1a."""
    from kpamd import catalog
    base = dict(next(r for r in catalog.load_ec2_table() if r["name"] == "m5.large"))
    base.update(name="test", vcpu=2, memory_mib=8192, arch="amd64", max_enis=3, ipv4_per_eni=10, eni_source="ec2",
                trunking=0, branch_enis=0, gpu_name="", gpu_manufacturer="", gpu_count=0, gpu_memory_mib="",
                accel_name="", accel_manufacturer="", accel_count=0, neuron_devices=0, neuron_cores_per_device=0,
                efa=0, local_nvme_gb="")
    return base


@pytest.mark.parametrize("backend", BACKENDS)
def test_windows_private_ipv4_launch(backend, mk, lib):
    """windows2022 nodeclass, a pod requesting one vpc.amazonaws.com/PrivateIPv4Address: scheduled, on a type the limits
    table advertises (IPv4PerInterface != 0) (R:suite_test.go:639-654)."""
    import scenarios
    from kpamd import catalog
    types = scenarios.fake_catalog(lib, ami_family="Windows2022")
    env = mk(backend, types)
    nodes, pod_node = env.provision([NodePool("default", 0, 0, OD_POOL)], [PodShape(rq(**{PIP: 1000}))], [1])
    assert pod_node == [0]
    row = {r["name"]: r for r in catalog.load_ec2_table()}[nodes[0]["type"]]
    assert row["eni_source"] == "vpclimits" and row["ipv4_per_eni"] > 0
    it = next(t for t in types if t.name == nodes[0]["type"])
    assert ("kubernetes.io/os", "In", ["windows"]) in [tuple(r[:3]) for r in it.requirements]


@pytest.mark.parametrize("backend", BACKENDS)
def test_windows_private_ipv4_not_advertised(backend, mk, lib):
    """The "test" type has IPv4 addresses but is not in the limits table: a pod requesting PrivateIPv4Address on a NodePool
    restricted to it stays pending (R:suite_test.go:655-706)."""
    import scenarios
    types = scenarios.fake_catalog(lib, ami_family="Windows2022", extra_rows=[(_test_type_row(), ["test-zone-1a"])])
    env = mk(backend, types)
    pool = [NodePool("default", 0, 0, OD_POOL + [(IT, "In", ["test"])])]
    _, pod_node = env.provision(pool, [PodShape(rq(**{PIP: 1000}))], [1])
    assert pod_node == [None]
    _, pod_node = env.provision(pool, [PodShape(rq())], [1])  # the type itself is launchable
    assert pod_node == [0]
