"""Pod anti-affinity and pod affinity on the hostname and on label keys such as the zone (ABI v6): upstream TopologyGroup of TopologyTypePodAntiAffinity
(nextDomainAntiAffinity: only domains whose count is zero; Topology.Record counts every selected pod on its node),
the inverse groups a bound pod's required terms create (Topology.updateInverseAntiAffinity: pods the selector selects
avoid the bound pod's node), TopologyTypePodAffinity (nextDomainAffinity: a node holding a selected pod, or — while no
domain has one and the pod selects itself — any node: the bootstrap), and Preferences.Relax's
removePreferredPodAffinityTerm / removePreferredPodAntiAffinityTerm (heaviest first, before the preferred
node-affinity terms). Docs: R:website/content/en/preview/concepts/scheduling.md:395-428 (the anti-affinity
example "avoid running on any node with a pod labeled app=inflate": one replica per node). A namespaceSelector adds
the cluster namespaces whose labels it matches (upstream Topology.buildNamespaceList; ABI v8: kp_solve_in.namespaces),
docs R:website/content/en/preview/concepts/scheduling.md:394-428.

Known answers on the CPU oracle, device == oracle under -m gpu (Solve and consolidation simulations). Parity
unpinned beyond the written semantics (upstream core is not in the container)."""
import copy
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from test_hostports_volumes import POOL_REQS, small_problem  # noqa: E402

HOST = "kubernetes.io/hostname"


def anti(app, weight=0, key=HOST, namespaces=()):
    from kpamd.model import LabelSelector, PodAffinityTerm
    return PodAffinityTerm(key, LabelSelector({"app": app}), list(namespaces), weight)


def shape(app, cpu_m=500, mem_mi=512, req=(), pref=(), **kw):
    from kpamd import synth
    from kpamd.model import PodShape
    return PodShape(synth.req_res(cpu_m, mem_mi), labels={"app": app}, required_anti_affinity=list(req),
                    preferred_anti_affinity=list(pref), **kw)


def oracle(prob):
    from oracle import pyoracle
    return pyoracle.solve(prob)


def m5_node(catalog, name="node-a"):
    from kpamd import synth
    from kpamd.model import ExistingNode
    it = catalog[[i for i, t in enumerate(catalog) if t.name == "m5.xlarge"][0]]
    return ExistingNode(name, synth.node_labels(it, 0, "on-demand", "default", name), it.allocatable())


# ---- oracle known answers (CPU) -------------------------------------------------------------------------------
def test_one_replica_per_node(catalog):
    r = oracle(small_problem(catalog, [shape("web", req=[anti("web")])], [5]))
    assert len(r["nodeclaims"]) == 5
    assert sorted(r["placement"].tolist()) == [0, 1, 2, 3, 4]


def test_selector_not_matching_itself(catalog):
    r = oracle(small_problem(catalog, [shape("web", req=[anti("db")])], [5]))
    assert len(r["nodeclaims"]) == 1


def test_other_pods_share(catalog):
    # web pods spread one per node; db pods (no terms) fill in beside them
    r = oracle(small_problem(catalog, [shape("web", 1000, 1024, req=[anti("web")]), shape("db", 250, 256)], [3, 6]))
    pl = r["placement"].tolist()
    assert len(set(pl[:3])) == 3
    assert set(pl[3:]) <= set(pl[:3])


def test_existing_node_with_selected_pod(catalog):
    node = m5_node(catalog)
    prob = small_problem(catalog, [shape("web", req=[anti("web")]), shape("api")], [1, 1], existing=[node])
    prob.bound_pods = [("default", {"app": "web"}, 0)]
    pl = oracle(prob)["placement"].tolist()
    assert pl[0] >= 0   # a web pod already runs on node-a
    assert pl[1] == -2  # no terms: the existing node


def test_inverse_anti_affinity_of_a_bound_pod(catalog):
    # the bound pod on node-a refuses company from app=web: a web pod without terms of its own avoids node-a
    node = m5_node(catalog)
    prob = small_problem(catalog, [shape("web"), shape("api")], [1, 1], existing=[node])
    prob.bound_pods = [("default", {"app": "cache"}, 0, [anti("web")])]
    pl = oracle(prob)["placement"].tolist()
    assert pl[0] >= 0 and pl[1] == -2


def test_namespaces(catalog):
    # the term selects app=web in namespace "other" only: default-namespace web pods are not counted
    r = oracle(small_problem(catalog, [shape("web", req=[anti("web", namespaces=["other"])])], [4]))
    assert len(r["nodeclaims"]) == 1


def test_preferred_term_relaxed_when_it_cannot_hold(catalog):
    # a cpu limit allows two NodeClaims: the third web pod fails with its preferred term, which Relax drops, and
    # it then joins one of the two
    from kpamd.model import NodePool
    prob = small_problem(catalog, [shape("web", 1000, 1024, pref=[anti("web", 50)])], [3])
    prob.nodepools = [NodePool("default", 0, 0, list(POOL_REQS) +
                               [("karpenter.k8s.aws/instance-cpu", "In", ["4"])], limits={"cpu": 8000})]
    pl = oracle(prob)["placement"].tolist()
    assert pl[0] != pl[1] and pl[2] in (pl[0], pl[1])


def aff(app, weight=0):
    from kpamd.model import LabelSelector, PodAffinityTerm
    return PodAffinityTerm(HOST, LabelSelector({"app": app}), [], weight)


def test_affinity_colocates_with_a_bound_pod(catalog):
    node = m5_node(catalog)
    prob = small_problem(catalog, [shape("web", required_affinity=[aff("cache")])], [2], existing=[node])
    prob.bound_pods = [("default", {"app": "cache"}, 0)]
    assert oracle(prob)["placement"].tolist() == [-2, -2]


def test_affinity_bootstrap_and_follow(catalog):
    # self-selecting: the first pod bootstraps (any node), the others must join a node holding one
    r = oracle(small_problem(catalog, [shape("web", required_affinity=[aff("web")])], [3]))
    assert r["placement"].tolist() == [0, 0, 0]


def test_affinity_without_target_fails(catalog):
    r = oracle(small_problem(catalog, [shape("web", required_affinity=[aff("cache")])], [2]))
    assert r["placement"].tolist() == [-1, -1]


def test_preferred_affinity_relaxed(catalog):
    r = oracle(small_problem(catalog, [shape("web", preferred_affinity=[aff("cache", 10)])], [2]))
    assert r["placement"].tolist() == [0, 0]


ZONE = "topology.kubernetes.io/zone"


def zaff(app, weight=0):
    from kpamd.model import LabelSelector, PodAffinityTerm
    return PodAffinityTerm(ZONE, LabelSelector({"app": app}), [], weight)


def zone_of(r, nc):
    return [q[2] for q in r["nodeclaims"][nc]["requirements"] if q[0] == ZONE]


def test_zone_anti_affinity(catalog):
    # pods pinned to a zone each: one per zone, a second pod for zone 1a has no zone left
    shapes = [shape("web", req=[anti("web", key=ZONE)], node_selector={ZONE: z})
              for z in ("test-zone-1a", "test-zone-1b", "test-zone-1c", "test-zone-1a")]
    pl = oracle(small_problem(catalog, shapes, [1, 1, 1, 1]))["placement"].tolist()
    assert len(set(pl[:3])) == 3 and min(pl[:3]) >= 0 and pl[3] == -1
    # unpinned: the first NodeClaim may launch in any zone, and Topology.Record blocks every zone it could be in
    # (for anti-affinity upstream records all of the node's possible domains), so the second pod has none left
    pl = oracle(small_problem(catalog, [shape("web", req=[anti("web", key=ZONE)])], [2]))["placement"].tolist()
    assert pl == [0, -1]


def test_zone_affinity_follows_the_first(catalog):
    # the self-selecting bootstrap pins the first NodeClaim to the lowest zone; the rest follow into that zone
    r = oracle(small_problem(catalog, [shape("web", required_affinity=[zaff("web")]), shape("api", required_affinity=[zaff("web")])], [2, 2]))
    zs = {tuple(zone_of(r, nc)[0]) for nc in set(r["placement"].tolist())}
    assert zs == {("test-zone-1a",)}


NAMESPACES = {"team-a": {"team": "a", "env": "prod"}, "team-b": {"team": "b", "env": "prod"},
              "sandbox": {"env": "dev"}, "default": {}}


def nsanti(app, nsel, namespaces=(), key=HOST, weight=0):
    """An anti-affinity term with a namespaceSelector (LabelSelector; {} = every namespace)."""
    from kpamd.model import LabelSelector, PodAffinityTerm
    sel = LabelSelector(dict(nsel)) if isinstance(nsel, dict) else nsel
    return PodAffinityTerm(key, LabelSelector({"app": app}), list(namespaces), weight, namespace_selector=sel)


def _ns_problem(catalog, term, bound_ns, pod_ns="default"):
    """node-a runs one bound app=web pod in namespace bound_ns; a new pod (namespace pod_ns) carries `term`."""
    node = m5_node(catalog)
    sh = shape("api", req=[term])
    sh.namespace = pod_ns
    prob = small_problem(catalog, [sh], [1], existing=[node])
    prob.bound_pods = [(bound_ns, {"app": "web"}, 0)]
    prob.namespaces = dict(NAMESPACES)
    return prob


@pytest.mark.parametrize("nsel,bound_ns,avoids", [
    ({"team": "a"}, "team-a", True),      # the selector picks team-a, where the web pod runs: node-a is avoided
    ({"team": "b"}, "team-a", False),     # picks team-b only: the team-a pod is not counted
    ({}, "sandbox", True),                # an empty selector selects every namespace
    ({"env": "prod"}, "sandbox", False),  # prod namespaces only
])
def test_namespace_selector(catalog, nsel, bound_ns, avoids):
    pl = oracle(_ns_problem(catalog, nsanti("web", nsel), bound_ns))["placement"].tolist()
    assert (pl[0] >= 0) == avoids and (pl[0] == -2) == (not avoids)


def test_namespace_selector_adds_to_listed_namespaces(catalog):
    # namespaces ["sandbox"] plus the selector's team-b: a web pod in sandbox is counted, one in team-a is not
    assert oracle(_ns_problem(catalog, nsanti("web", {"team": "b"}, ["sandbox"]), "sandbox"))["placement"][0] >= 0
    assert oracle(_ns_problem(catalog, nsanti("web", {"team": "b"}, ["sandbox"]), "team-a"))["placement"][0] == -2


def test_namespace_selector_expressions_and_own_namespace(catalog):
    # a selector given: the pod's own namespace is not implied (upstream buildNamespaceList)
    from kpamd.model import LabelSelector
    sel = LabelSelector({}, [("team", "In", ["a", "b"])])
    assert oracle(_ns_problem(catalog, nsanti("web", sel), "default", pod_ns="default"))["placement"][0] == -2
    assert oracle(_ns_problem(catalog, nsanti("web", sel), "team-b"))["placement"][0] >= 0
    sel = LabelSelector({}, [("team", "DoesNotExist", [])])
    assert oracle(_ns_problem(catalog, nsanti("web", sel), "sandbox"))["placement"][0] >= 0


def test_namespace_selector_host_compile(catalog):
    import kpamd
    assert kpamd.validate(_ns_problem(catalog, nsanti("web", {"team": "a"}), "team-a")) == 0
    assert kpamd.validate(small_problem(catalog, [shape("web", req=[anti("web")])], [2])) == 0


# ---- randomized (oracle on CPU, device under -m gpu) --------------------------------------------------------------
def add_anti(prob, seed, p=0.4):
    rng = np.random.default_rng(seed)
    prob = copy.deepcopy(prob)
    prob.namespaces = dict(NAMESPACES)
    apps = [f"app-{i}" for i in range(4)]
    for i, sh in enumerate(prob.shapes):
        sh.labels = dict(sh.labels or {}, app=apps[i % 4])
        if rng.random() < p:
            sh.required_anti_affinity = [anti(str(rng.choice(apps)), key=str(rng.choice([HOST, HOST, ZONE])))]
        if rng.random() < 0.2:
            sh.preferred_anti_affinity = [anti(str(rng.choice(apps)), int(rng.integers(1, 100)))
                                          for _ in range(int(rng.integers(1, 3)))]
        if rng.random() < 0.15:
            sh.required_affinity = [aff(str(rng.choice(apps))) if rng.random() < 0.6 else zaff(str(rng.choice(apps)))]
        if rng.random() < 0.15:
            sh.preferred_affinity = [aff(str(rng.choice(apps)), int(rng.integers(1, 100)))]
    bound = []
    for e in range(len(prob.existing)):
        for _ in range(int(rng.integers(0, 3))):
            terms = [anti(str(rng.choice(apps)))] if rng.random() < 0.3 else []
            bound.append(("default", {"app": str(rng.choice(apps))}, e, terms))
    prob.bound_pods = bound
    # namespaces and namespaceSelectors (a separate stream: the draws above stay as they were)
    r2 = np.random.default_rng(seed + 1000)
    nss, sels = sorted(NAMESPACES), [{"team": "a"}, {}, {"env": "prod"}, {"team": "b"}]
    for sh in prob.shapes:
        sh.namespace = str(r2.choice(nss))
        sh.required_anti_affinity = [nsanti(t.selector.match_labels["app"], sels[int(r2.integers(len(sels)))],
                                            key=t.topology_key) if r2.random() < 0.5 else t
                                     for t in (sh.required_anti_affinity or [])]
    prob.bound_pods = [(str(r2.choice(nss)), lab, e, terms) for _, lab, e, terms in prob.bound_pods]
    return prob


@pytest.mark.parametrize("seed", range(3))
def test_random_oracle_and_host_compile(catalog, seed):
    import kpamd
    from kpamd import synth
    prob = add_anti(synth.random_problem(catalog, 500 + seed, n_types=120, n_pods=200, n_pools=3,
                                         n_existing=[0, 10][seed % 2], n_shapes=14), seed)
    r = oracle(prob)
    assert len(r["placement"]) == prob.n_pods
    assert kpamd.validate(prob) == 0


@pytest.mark.gpu
def test_gpu_known_answers(ctx, catalog):
    import kpamd
    from test_gpu_parity import check_same
    from kpamd.model import NodePool
    node = m5_node(catalog)
    probs = [small_problem(catalog, [shape("web", req=[anti("web")])], [5]),
             small_problem(catalog, [shape("web", 1000, 1024, req=[anti("web")]), shape("db", 250, 256)], [3, 6])]
    p = small_problem(catalog, [shape("web", req=[anti("web")]), shape("api")], [1, 1], existing=[node])
    p.bound_pods = [("default", {"app": "web"}, 0)]
    probs.append(p)
    p = small_problem(catalog, [shape("web"), shape("api")], [1, 1], existing=[m5_node(catalog)])
    p.bound_pods = [("default", {"app": "cache"}, 0, [anti("web")])]
    probs.append(p)
    p = small_problem(catalog, [shape("web", 1000, 1024, pref=[anti("web", 50)])], [3])
    p.nodepools = [NodePool("default", 0, 0, list(POOL_REQS) + [("karpenter.k8s.aws/instance-cpu", "In", ["4"])],
                            limits={"cpu": 8000})]
    probs.append(p)
    p = small_problem(catalog, [shape("web", required_affinity=[aff("cache")])], [2], existing=[m5_node(catalog)])
    p.bound_pods = [("default", {"app": "cache"}, 0)]
    probs += [p, small_problem(catalog, [shape("web", required_affinity=[aff("web")])], [3]),
              small_problem(catalog, [shape("web", required_affinity=[aff("cache")])], [2]),
              small_problem(catalog, [shape("web", preferred_affinity=[aff("cache", 10)])], [2]),
              small_problem(catalog, [shape("web", req=[anti("web", key=ZONE)], node_selector={ZONE: z})
                                      for z in ("test-zone-1a", "test-zone-1b", "test-zone-1c", "test-zone-1a")],
                            [1, 1, 1, 1]),
              small_problem(catalog, [shape("web", req=[anti("web", key=ZONE)])], [2]),
              small_problem(catalog, [shape("web", required_affinity=[zaff("web")]),
                                      shape("api", required_affinity=[zaff("web")])], [2, 2])]
    for prob in probs:
        check_same(kpamd.Scheduler(ctx, prob).solve(), oracle(prob))


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(8))
def test_gpu_random_anti_affinity(ctx, catalog, seed):
    import kpamd
    from kpamd import synth
    from test_gpu_parity import check_same
    prob = add_anti(synth.random_problem(catalog, 600 + seed, n_types=150, n_pods=300, n_pools=3,
                                         n_existing=[0, 6, 30][seed % 3], n_shapes=18), seed)
    check_same(kpamd.Scheduler(ctx, prob).solve(), oracle(prob))


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(3))
def test_gpu_consolidation_anti_affinity(ctx, catalog, seed, general_mode):
    from kpamd import synth
    from test_gpu_consolidation import check
    cl = synth.random_cluster(catalog, 70 + seed, n_nodes=[20, 30, 40][seed])
    rng = np.random.default_rng(seed)
    for i, sh in enumerate(cl.shapes):
        sh.labels = {"app": f"app-{i % 4}"}
        if rng.random() < 0.4:
            sh.required_anti_affinity = [anti(f"app-{int(rng.integers(0, 4))}")]
        elif rng.random() < 0.2:
            sh.preferred_affinity = [aff(f"app-{int(rng.integers(0, 4))}", 5)]
    subs = synth.consolidation_subsets(cl, 15, seed=seed, max_size=min(12, len(cl.nodes)))
    subs += [[c] for c in cl.candidates[:10]]
    check(ctx, cl, subs, multi_node=bool(seed % 2))


@pytest.mark.gpu
def test_gpu_namespace_selector(ctx, catalog):
    """namespaceSelector on the device (host compile resolves the namespaces) == the oracle."""
    import kpamd
    from kpamd.model import LabelSelector
    from test_gpu_parity import check_same
    cases = [({"team": "a"}, "team-a"), ({"team": "b"}, "team-a"), ({}, "sandbox"), ({"env": "prod"}, "sandbox"),
             (LabelSelector({}, [("team", "In", ["a", "b"])]), "team-b")]
    for nsel, bound_ns in cases:
        prob = _ns_problem(catalog, nsanti("web", nsel), bound_ns)
        check_same(kpamd.Scheduler(ctx, prob).solve(), oracle(prob))
