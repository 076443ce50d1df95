"""Pod requirements on kubernetes.io/hostname (nodeSelector, required and preferred node affinity).

Upstream semantics restated: every NodeClaim carries `hostname In {a unique placeholder}`
(NewNodeClaim), every existing node `hostname In {its hostname}` (NewExistingNode: the label, else the node name), so
a pod's hostname requirement admits exactly the existing nodes it names (In), all but those (NotIn), any node
(Exists) or none (DoesNotExist); a NodeClaim admits NotIn / Exists only. The product restates the values with two
dictionary stand-ins (the names no pod mentions, the NodeClaims' placeholder); the CPU oracle keeps the literal
values. KATs on the oracle (CPU) and the device (-m gpu, which must equal the oracle); randomized problems and a
consolidation cluster (general path) compare device and oracle. The reference's own tests use hostname only as a
topology key: parity with upstream is unpinned beyond the written semantics.
"""
import numpy as np
import pytest

HOST = "kubernetes.io/hostname"
BACKENDS = ["oracle", pytest.param("device", marks=pytest.mark.gpu)]


def _node(catalog, name, tname="m5.xlarge", zone="test-zone-1a", label=True, used_cpu=0):
    from kpamd.model import ExistingNode
    it = next(t for t in catalog if t.name == tname)
    labels = {"node.kubernetes.io/instance-type": tname, "topology.kubernetes.io/zone": zone,
              "karpenter.sh/capacity-type": "on-demand", "kubernetes.io/arch": "amd64", "kubernetes.io/os": "linux"}
    if label:
        labels[HOST] = name
    alloc = it.allocatable()
    return ExistingNode(name, labels, dict(alloc), {"cpu": used_cpu, "pods": 0})


def _problem(catalog, shapes, counts, existing):
    from kpamd.model import NodePool, Problem
    import scenarios
    pool = NodePool("default", 0, 0, [("karpenter.sh/capacity-type", "In", ["on-demand"])])
    s, c, u = scenarios.pods_of(counts)
    return Problem([catalog], [pool], shapes, s, c, u, existing=existing, name="hostname")


def _solve(request, backend, prob):
    from oracle import pyoracle
    want = pyoracle.solve(prob)
    if backend == "oracle":
        return want
    import kpamd
    from test_gpu_parity import check_same
    got = kpamd.Scheduler(request.getfixturevalue("ctx"), prob).solve()
    check_same(got, want)
    return got


@pytest.mark.parametrize("backend", BACKENDS)
def test_hostname_selectors(request, catalog, backend):
    from kpamd import synth
    from kpamd.model import PodShape
    nodes = [_node(catalog, "node-a"), _node(catalog, "node-c", label=False)]
    shapes = [PodShape(synth.req_res(500, 512), node_selector={HOST: "node-a"}),          # -> node-a
              PodShape(synth.req_res(500, 512), node_selector={HOST: "node-b"}),          # no such node: pending
              PodShape(synth.req_res(500, 512), required_terms=[[(HOST, "NotIn", ["node-a", "node-c"])]]),  # new
              PodShape(synth.req_res(500, 512), required_terms=[[(HOST, "In", ["node-c"])]]),  # the name, no label
              PodShape(synth.req_res(500, 512), required_terms=[[(HOST, "DoesNotExist", [])]]),  # nowhere
              PodShape(synth.req_res(500, 512), required_terms=[[(HOST, "Exists", [])]])]  # first existing node
    res = _solve(request, backend, _problem(catalog, shapes, [2, 1, 1, 1, 1, 1], nodes))
    pl = list(res["placement"])
    assert pl[0] == pl[1] == -2 and pl[2] == -1 and pl[3] >= 0 and pl[4] == -3 and pl[5] == -1 and pl[6] == -2
    assert all(HOST not in [r[0] for r in n["requirements"]] for n in res["nodeclaims"])


@pytest.mark.parametrize("backend", BACKENDS)
def test_preferred_hostname_relaxes(request, catalog, backend):
    """A preferred hostname term whose node is full relaxes onto a new NodeClaim."""
    from kpamd import synth
    from kpamd.model import PodShape
    full = _node(catalog, "node-a", used_cpu=4000)  # m5.xlarge: 4 vCPU allocatable minus overhead: no room
    shapes = [PodShape(synth.req_res(1000, 512), preferred_terms=[(50, [(HOST, "In", ["node-a"])])])]
    res = _solve(request, backend, _problem(catalog, shapes, [2], [full]))
    assert all(p >= 0 for p in res["placement"])


def _random(catalog, seed):
    from kpamd import synth
    rng = np.random.default_rng(seed)
    prob = synth.random_problem(catalog, 900 + seed, n_types=100, n_pods=250, n_pools=2, n_existing=12, n_shapes=16)
    names = [e.name for e in prob.existing]
    for e in prob.existing[::2]:
        e.labels = dict(e.labels, **{HOST: e.name})
    for sh in prob.shapes:
        u = rng.random()
        pick = [str(x) for x in rng.choice(names + ["ghost"], size=2, replace=False)]
        if u < 0.2:
            sh.node_selector = dict(sh.node_selector or {}, **{HOST: pick[0]})
        elif u < 0.4:
            sh.required_terms = [list(t) + [(HOST, "NotIn", pick)] for t in (sh.required_terms or [[]])]
        elif u < 0.55:
            sh.preferred_terms = list(sh.preferred_terms or []) + [(int(rng.integers(1, 100)), [(HOST, "In", pick)])]
    return prob


@pytest.mark.parametrize("seed", range(3))
def test_random_hostname_oracle_and_host_compile(catalog, seed):
    import kpamd
    from oracle import pyoracle
    prob = _random(catalog, seed)
    assert len(pyoracle.solve(prob)["placement"]) == prob.n_pods
    assert kpamd.validate(prob) == 0


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(6))
def test_gpu_random_hostname(ctx, catalog, seed):
    import kpamd
    from oracle import pyoracle
    from test_gpu_parity import check_same
    prob = _random(catalog, seed)
    check_same(kpamd.Scheduler(ctx, prob).solve(), pyoracle.solve(prob))


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(2))
def test_gpu_hostname_consolidation(ctx, catalog, seed, general_mode):
    """A cluster whose pods pin hostnames takes the general path (the batched sim kernels drop the hostname)."""
    from kpamd import synth
    from test_gpu_consolidation import check
    cl = synth.random_cluster(catalog, 80 + seed, n_nodes=24)
    for n in cl.nodes:
        n.node.labels = dict(n.node.labels, **{HOST: n.node.name})
    cl.shapes[0].required_terms = [[(HOST, "NotIn", [cl.nodes[0].node.name, cl.nodes[1].node.name])]]
    cl.shapes[1].preferred_terms = [(10, [(HOST, "In", [cl.nodes[2].node.name])])]
    subs = synth.consolidation_subsets(cl, 12, seed=seed, max_size=8) + [[c] for c in cl.candidates[:8]]
    check(ctx, cl, subs, multi_node=bool(seed % 2))
