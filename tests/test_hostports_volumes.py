"""Host ports (upstream scheduling.HostPortUsage, checked by NodeClaim.Add and ExistingNode.CanAdd) and volume
topology (upstream VolumeTopology.Inject: the pod's volume requirements appended to every required node-affinity
term) — ABI v6.

Known-answer cases on the CPU oracle follow the upstream semantics (hostportusage.go: hostIP "" = 0.0.0.0, protocol
"" = TCP, hostPort 0 skipped, Matches = same protocol + port and an unspecified IP on either side or equal IPs;
volumetopology.go Inject). The reference repo holds no host-port fixture (its e2e storage suite,
R:test/suites/storage/suite_test.go:109-200, asserts "one node, pod healthy" for zonal PVs and StorageClass
allowedTopologies on topology.ebs.csi.aws.com/zone, which karpv1.NormalizedLabels maps to the zone label,
R:pkg/operator/operator.go:71): those two cases are restated here; the rest is parity unpinned beyond the written
semantics. Under -m gpu the device path must equal the oracle bit-exactly on the same inputs, Solve and
consolidation simulations.
"""
import copy
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

ZONE = "topology.kubernetes.io/zone"
POOL_REQS = [("karpenter.sh/capacity-type", "In", ["on-demand"]),
             ("karpenter.k8s.aws/instance-category", "In", ["c", "m", "r"]),
             ("karpenter.k8s.aws/instance-generation", "Gt", ["4"])]


def small_problem(catalog, shapes, counts, existing=(), name="hp"):
    from kpamd.model import NodePool, Problem
    shape = np.concatenate([np.full(c, i, np.uint32) for i, c in enumerate(counts)])
    n = len(shape)
    return Problem([catalog], [NodePool("default", 0, 0, list(POOL_REQS))], shapes, shape,
                   np.full(n, 1_750_000_000, np.int64) + np.arange(n), np.arange(n, dtype=np.uint64) + 1,
                   existing=list(existing), name=name)


def shape(cpu_m=500, mem_mi=512, ports=(), vol=(), **kw):
    from kpamd import synth
    from kpamd.model import PodShape
    return PodShape(synth.req_res(cpu_m, mem_mi), host_ports=list(ports), volume_requirements=list(vol), **kw)


def oracle(prob):
    from oracle import pyoracle
    return pyoracle.solve(prob)


def nodeclaims_of(res, pods):
    return sorted({int(res["placement"][p]) for p in pods})


# ---- oracle known answers (CPU) -------------------------------------------------------------------------------
def test_same_port_one_pod_per_nodeclaim(catalog):
    prob = small_problem(catalog, [shape(ports=[(None, 80, "TCP")])], [5])
    r = oracle(prob)
    assert len(r["nodeclaims"]) == 5
    assert sorted(r["placement"].tolist()) == [0, 1, 2, 3, 4]


def test_distinct_ports_and_protocols_share(catalog):
    shapes = [shape(ports=[(None, 80, "TCP")]), shape(ports=[(None, 80, "UDP")]), shape(ports=[("", 443, None)]),
              shape(ports=[(None, 0, "TCP")]), shape(ports=[(None, 0, "TCP")])]  # hostPort 0: not a host port
    r = oracle(small_problem(catalog, shapes, [1, 1, 1, 1, 1]))
    assert len(r["nodeclaims"]) == 1


def test_specific_ips(catalog):
    # 10.0.0.1:80 and 10.0.0.2:80 coexist; ::ffff:10.0.0.1 is the same IP (net.IP.Equal); 0.0.0.0:80 matches all
    shapes = [shape(ports=[("10.0.0.1", 80, "TCP")]), shape(ports=[("10.0.0.2", 80, "TCP")]),
              shape(ports=[("::ffff:10.0.0.1", 80, "TCP")]), shape(ports=[("0.0.0.0", 80, "TCP")])]
    r = oracle(small_problem(catalog, shapes, [1, 1, 1, 1]))
    pl = r["placement"]
    assert pl[0] == pl[1]
    assert pl[2] != pl[0]
    assert pl[3] not in (pl[0], pl[2])
    assert len(r["nodeclaims"]) == 3


def test_existing_node_ports(catalog):
    from kpamd import synth
    from kpamd.model import ExistingNode
    it = catalog[[i for i, t in enumerate(catalog) if t.name == "m5.xlarge"][0]]
    labels = synth.node_labels(it, 0, "on-demand", "default", "node-a")
    node = ExistingNode("node-a", labels, it.allocatable(), host_ports=[(None, 80, "TCP")])
    shapes = [shape(ports=[(None, 80, "TCP")]), shape(), shape(ports=[(None, 8080, "TCP")])]
    r = oracle(small_problem(catalog, shapes, [1, 1, 2], existing=[node]))
    pl = r["placement"].tolist()
    assert pl[0] >= 0          # port 80 is taken on the node: a new NodeClaim
    assert pl[1] == -2         # no ports: the existing node
    assert pl[2] == -2 and pl[3] >= 0  # 8080: the first takes the node, the second conflicts with it


def test_volume_zone_requirement(catalog):
    # zonal PV (R:test/suites/storage/suite_test.go:109-127) and StorageClass allowedTopologies on the EBS CSI key
    # (:180-200): the NodeClaim lands in that zone
    for key in (ZONE, "topology.ebs.csi.aws.com/zone"):
        r = oracle(small_problem(catalog, [shape(vol=[(key, "In", ["test-zone-1b"])])], [3]))
        assert len(r["nodeclaims"]) == 1
        zreq = [q for q in r["nodeclaims"][0]["requirements"] if q[0] == ZONE]
        assert zreq and zreq[0][2] == ["test-zone-1b"], r["nodeclaims"][0]["requirements"]


def test_volume_requirement_joins_every_term(catalog):
    # two required terms (ORed): the volume's zone is appended to both; a node selector on another zone conflicts
    s1 = shape(vol=[(ZONE, "In", ["test-zone-1c"])],
               required_terms=[[("karpenter.k8s.aws/instance-category", "In", ["c"])],
                               [("karpenter.k8s.aws/instance-category", "In", ["m"])]])
    s2 = shape(vol=[(ZONE, "In", ["test-zone-1c"])], node_selector={ZONE: "test-zone-1a"})
    r = oracle(small_problem(catalog, [s1, s2], [1, 1]))
    pl = r["placement"].tolist()
    assert pl[0] >= 0 and pl[1] == -1
    reqs = dict((q[0], q[2]) for q in r["nodeclaims"][pl[0]]["requirements"])
    assert reqs[ZONE] == ["test-zone-1c"]


def test_invalid_host_ip_is_inval(catalog):
    import kpamd
    from oracle import pyoracle
    prob = small_problem(catalog, [shape(ports=[("not-an-ip", 80, "TCP")])], [1])
    with pytest.raises(RuntimeError):
        pyoracle.solve(prob)
    rc = kpamd.validate(prob) if hasattr(kpamd, "validate") else None
    if rc is not None:
        assert rc == kpamd.abi.KP_E_INVAL


# ---- randomized scenarios (oracle on CPU, device under -m gpu) ----------------------------------------------------
PORTS = [(None, 80, "TCP"), ("10.0.0.1", 80, "TCP"), ("10.0.0.2", 80, "TCP"), ("::ffff:10.0.0.2", 80, "TCP"),
         (None, 80, "UDP"), (None, 443, "TCP"), ("10.0.0.1", 9100, "TCP"), (None, 0, "TCP")]


def add_ports_and_volumes(prob, seed, p_ports=0.35, p_vol=0.2):
    from kpamd import synth
    rng = np.random.default_rng(seed)
    prob = copy.deepcopy(prob)
    for sh in prob.shapes:
        if rng.random() < p_ports:
            k = int(rng.integers(1, 3))
            sh.host_ports = [PORTS[i] for i in rng.choice(len(PORTS), size=k, replace=False)]
        if rng.random() < p_vol:
            sh.volume_requirements = [(ZONE, "In", list(rng.choice(synth.ZONES, size=int(rng.integers(1, 3)),
                                                                    replace=False)))]
    for n in prob.existing:
        if rng.random() < 0.4:
            n.host_ports = [PORTS[int(rng.integers(0, len(PORTS)))]]
    return prob


@pytest.mark.parametrize("seed", range(4))
def test_random_oracle_runs(catalog, seed):
    from kpamd import synth
    prob = add_ports_and_volumes(synth.random_problem(catalog, seed, n_types=120, n_pods=200, n_pools=3,
                                                      n_existing=[0, 8][seed % 2], n_shapes=16), seed)
    r = oracle(prob)
    assert len(r["placement"]) == prob.n_pods


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(10))
def test_gpu_random_host_ports_volumes(ctx, catalog, seed):
    import kpamd
    from kpamd import synth
    from test_gpu_parity import check_same
    prob = add_ports_and_volumes(synth.random_problem(catalog, 300 + seed, n_types=150, n_pods=300, n_pools=3,
                                                      n_existing=[0, 6, 30][seed % 3], n_shapes=20), seed)
    got = kpamd.Scheduler(ctx, prob).solve()
    check_same(got, oracle(prob))


@pytest.mark.gpu
def test_gpu_known_answers(ctx, catalog):
    import kpamd
    from test_gpu_parity import check_same
    from kpamd import synth
    from kpamd.model import ExistingNode
    it = catalog[[i for i, t in enumerate(catalog) if t.name == "m5.xlarge"][0]]
    node = ExistingNode("node-a", synth.node_labels(it, 0, "on-demand", "default", "node-a"), it.allocatable(),
                        host_ports=[(None, 80, "TCP")])
    probs = [small_problem(catalog, [shape(ports=[(None, 80, "TCP")])], [5]),
             small_problem(catalog, [shape(ports=[("10.0.0.1", 80, "TCP")]), shape(ports=[("10.0.0.2", 80, "TCP")]),
                                     shape(ports=[("::ffff:10.0.0.1", 80, "TCP")]),
                                     shape(ports=[("0.0.0.0", 80, "TCP")])], [1, 1, 1, 1]),
             small_problem(catalog, [shape(ports=[(None, 80, "TCP")]), shape(), shape(ports=[(None, 8080, "TCP")])],
                           [1, 1, 2], existing=[node]),
             small_problem(catalog, [shape(vol=[("topology.ebs.csi.aws.com/zone", "In", ["test-zone-1b"])])], [3]),
             # a deployment with a host port mixed into config 2's shapes: fast lane and full path interleave
             add_ports_and_volumes(synth.config2(catalog, n_pods=2000, seed=11), 11, p_ports=0.1, p_vol=0.1)]
    for prob in probs:
        check_same(kpamd.Scheduler(ctx, prob).solve(), oracle(prob))


def cluster_with_ports(catalog, seed):
    from kpamd import synth
    cl = synth.random_cluster(catalog, seed, n_nodes=[20, 40][seed % 2])
    rng = np.random.default_rng(seed)
    for sh in cl.shapes:
        if rng.random() < 0.4:
            sh.host_ports = [PORTS[int(rng.integers(0, 7))]]
    for n in cl.nodes:
        if rng.random() < 0.2:
            n.node.host_ports = [PORTS[int(rng.integers(0, 7))]]
    return cl


def test_cluster_oracle_runs(catalog):
    from kpamd import synth
    from oracle import pyoracle
    cl = cluster_with_ports(catalog, 3)
    res, _ = pyoracle.simulate_batch(cl, synth.consolidation_subsets(cl, 10, seed=3, max_size=10))
    assert len(res) >= 10


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(4))
def test_gpu_consolidation_host_ports(ctx, catalog, seed):
    from kpamd import synth
    from test_gpu_consolidation import check
    cl = cluster_with_ports(catalog, seed)
    subs = synth.consolidation_subsets(cl, 25, seed=seed, max_size=min(30, len(cl.nodes)))
    subs += [[c] for c in cl.candidates[:15]]
    check(ctx, cl, subs, multi_node=bool(seed % 2))


def test_product_host_compile(catalog):
    """kp_solve_validate (host compile, no device): the randomized batches compile; > 64 distinct port entries in
    one batch is KP_E_UNSUPPORTED (the Go path runs)."""
    import kpamd
    from kpamd import synth
    for seed in range(4):
        prob = add_ports_and_volumes(synth.random_problem(catalog, seed, n_types=120, n_pods=200, n_pools=3,
                                                          n_existing=8, n_shapes=16), seed)
        assert kpamd.validate(prob) == 0
    many = [shape(ports=[(None, 1000 + i, "TCP")]) for i in range(65)]
    assert kpamd.validate(small_problem(catalog, many, [1] * 65)) == kpamd.abi.KP_E_UNSUPPORTED
