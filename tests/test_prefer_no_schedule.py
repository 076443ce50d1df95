"""PreferNoSchedule taints and upstream's last relaxation, `Preferences.toleratePreferNoScheduleTaints`.

Upstream semantics restated (UP pkg/controllers/provisioning/scheduling/{scheduler.go,preferences.go}):
* `Taints.ToleratesPod` treats a taint of every effect as hard, PreferNoSchedule included, for NodeClaims (the
  NodePool template's taints) and for existing nodes.
* `NewScheduler` sets `Preferences.ToleratePreferNoSchedule` when any NodePool template taint has effect
  PreferNoSchedule (NodePool taints may carry it: R:pkg/apis/crds/karpenter.sh_nodepools.yaml:344-348).
* With it set, `Relax` ends with `toleratePreferNoScheduleTaints`: after every other relaxation (required OR-terms,
  preferred pod (anti-)affinity, preferred node affinity, ScheduleAnyway spreads) it appends
  `{Operator: Exists, Effect: PreferNoSchedule}` unless a toleration already equals it (`MatchToleration`), and the
  pod is re-queued as relaxed. So a pod first avoids such a pool and lands there once nothing else takes it
  (relaxation model: R:website/content/en/preview/concepts/scheduling.md:212-216).

KATs on the oracle (CPU) and the device (-m gpu, equal to the oracle); randomized Solve problems, topology
problems and consolidation clusters with PreferNoSchedule pools / nodes compare device and oracle. The reference
holds no test of this relaxation: parity with upstream is unpinned beyond the written semantics.
"""
import numpy as np
import pytest

BACKENDS = ["oracle", pytest.param("device", marks=pytest.mark.gpu)]
PNS = "PreferNoSchedule"


def _pools(plain_limit_cpu=None, soft_weight=10, plain_zone=None, soft_taint=True):
    from kpamd.model import NodePool
    soft_reqs = [("karpenter.sh/capacity-type", "In", ["on-demand"]), ("node.kubernetes.io/instance-type", "In", ["m5.xlarge"])]
    plain_reqs = [("karpenter.sh/capacity-type", "In", ["on-demand"]), ("node.kubernetes.io/instance-type", "In", ["c5.xlarge"])]
    if plain_zone:
        plain_reqs.append(("topology.kubernetes.io/zone", "In", [plain_zone]))
        soft_reqs.append(("topology.kubernetes.io/zone", "NotIn", [plain_zone]))
    soft = NodePool("soft", soft_weight, 0, soft_reqs, taints=[("soft", "true", PNS)] if soft_taint else [])
    plain = NodePool("plain", 1, 0, plain_reqs, limits={"cpu": plain_limit_cpu} if plain_limit_cpu else {})
    return [soft, plain]


def _node(catalog, name, taints, used_cpu=0, tname="m5.2xlarge"):
    from kpamd.model import ExistingNode
    it = next(t for t in catalog if t.name == tname)
    labels = {"node.kubernetes.io/instance-type": tname, "topology.kubernetes.io/zone": "test-zone-1a",
              "karpenter.sh/capacity-type": "on-demand", "kubernetes.io/arch": "amd64", "kubernetes.io/os": "linux",
              "kubernetes.io/hostname": name}
    return ExistingNode(name, labels, dict(it.allocatable()), {"cpu": used_cpu, "pods": 0}, taints)


def _problem(catalog, pools, shapes, counts, existing=()):
    from kpamd.model import Problem
    import scenarios
    s, c, u = scenarios.pods_of(counts)
    return Problem([catalog], pools, shapes, s, c, u, existing=list(existing), name="prefer-no-schedule")


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


def _pools_of(res, pools):
    """NodePool name per pod: existing node 'node:<i>', pending None."""
    out = []
    for p in res["placement"]:
        p = int(p)
        if p >= 0:
            out.append(pools[res["nodeclaims"][p]["nodepool"]].name)
        elif p == -1:
            out.append(None)
        else:
            out.append(f"node:{-2 - p}")
    return out


@pytest.mark.parametrize("backend", BACKENDS)
def test_avoids_prefer_no_schedule_pool_while_another_fits(request, catalog, backend):
    """The heavier pool is tainted PreferNoSchedule: the pod skips it (a hard taint to ToleratesPod) and lands on
    the lighter, untainted pool without relaxing."""
    from kpamd import synth
    from kpamd.model import PodShape
    pools = _pools()
    res = _solve(request, backend, _problem(catalog, pools, [PodShape(synth.req_res(500, 512))], [3]))
    assert _pools_of(res, pools) == ["plain"] * 3


@pytest.mark.parametrize("backend", BACKENDS)
def test_relaxes_onto_prefer_no_schedule_pool_when_nothing_else_fits(request, catalog, backend):
    """The untainted pool's cpu limit admits one c5.xlarge (4 vCPU); the pods that no longer fit relax to tolerate
    PreferNoSchedule and land on the tainted pool."""
    from kpamd import synth
    from kpamd.model import PodShape
    pools = _pools(plain_limit_cpu=4000)
    res = _solve(request, backend, _problem(catalog, pools, [PodShape(synth.req_res(1500, 512))], [6]))
    got = _pools_of(res, pools)
    assert got[:2] == ["plain", "plain"]  # one c5.xlarge takes two 1.5-vCPU pods, then the limit binds
    assert got[2:] == ["soft"] * 4 and None not in got


@pytest.mark.parametrize("backend", BACKENDS)
def test_relaxation_is_last(request, catalog, backend):
    """toleratePreferNoScheduleTaints comes after removePreferredNodeAffinityTerm: a pod preferring the tainted
    pool's zone first drops the preference and lands on the untainted pool in another zone."""
    from kpamd import synth
    from kpamd.model import PodShape
    pools = _pools(plain_zone="test-zone-1b")
    sh = PodShape(synth.req_res(500, 512), preferred_terms=[(50, [("topology.kubernetes.io/zone", "In", ["test-zone-1a"])])])
    res = _solve(request, backend, _problem(catalog, pools, [sh], [2]))
    assert _pools_of(res, pools) == ["plain", "plain"]


@pytest.mark.parametrize("backend", BACKENDS)
def test_exact_toleration_goes_by_weight(request, catalog, backend):
    """A pod that already tolerates PreferNoSchedule (the exact toleration the relaxation would add, or a
    key-specific one) takes the heavier tainted pool first, by weight order."""
    from kpamd import synth
    from kpamd.model import PodShape
    pools = _pools()
    shapes = [PodShape(synth.req_res(500, 512), tolerations=[("", "Exists", "", PNS)]),
              PodShape(synth.req_res(400, 512), tolerations=[("soft", "Exists", "", PNS)]),
              PodShape(synth.req_res(300, 512), tolerations=[("soft", "Equal", "false", PNS)])]  # wrong value
    res = _solve(request, backend, _problem(catalog, pools, shapes, [1, 1, 1]))
    assert _pools_of(res, pools) == ["soft", "soft", "plain"]


@pytest.mark.parametrize("backend", BACKENDS)
def test_existing_node_prefer_no_schedule(request, catalog, backend):
    """Existing nodes: a PreferNoSchedule-tainted node is skipped at first; once the pod relaxes (a NodePool carries
    such a taint) it lands on that node, which existing-node placement tries before any NodeClaim."""
    from kpamd import synth
    from kpamd.model import PodShape
    pools = _pools(plain_limit_cpu=4000)
    nodes = [_node(catalog, "node-a", [("soft", "node", PNS)])]
    res = _solve(request, backend, _problem(catalog, pools, [PodShape(synth.req_res(1500, 512))], [4], nodes))
    got = _pools_of(res, pools)
    assert got[:2] == ["plain", "plain"] and got[2:] == ["node:0", "node:0"]


@pytest.mark.parametrize("backend", BACKENDS)
def test_no_relaxation_without_a_prefer_no_schedule_pool(request, catalog, backend):
    """No NodePool has a PreferNoSchedule taint: the relaxation is off, so a node tainted PreferNoSchedule stays
    hard for the pods, which end pending once the pool's limit binds."""
    from kpamd import synth
    from kpamd.model import PodShape
    pools = _pools(plain_limit_cpu=4000, soft_taint=False)
    pools[0].requirements = pools[0].requirements + [("karpenter.sh/capacity-type", "In", ["spot"])]  # soft: nothing
    nodes = [_node(catalog, "node-a", [("soft", "node", PNS)])]
    res = _solve(request, backend, _problem(catalog, pools, [PodShape(synth.req_res(1500, 512))], [4], nodes))
    assert _pools_of(res, pools) == ["plain", "plain", None, None]


@pytest.mark.parametrize("backend", BACKENDS)
def test_prefer_no_schedule_with_spread(request, catalog, backend):
    """A DoNotSchedule zone spread with nodeTaintsPolicy Honor: the relaxed level tolerates the taint, so its spread
    group is another group (the node filter carries the tolerations), counted from the cluster (Topology.Update)."""
    from kpamd import synth
    from kpamd.model import LabelSelector, PodShape, TopologySpread
    pools = _pools(plain_limit_cpu=4000)
    for p in pools:
        p.requirements = [r for r in p.requirements if r[0] != "node.kubernetes.io/instance-type"] + \
            [("node.kubernetes.io/instance-type", "In", ["m5.large", "c5.large"])]
    sh = PodShape(synth.req_res(1000, 512), labels={"app": "w"},
                  topology_spread=[TopologySpread("topology.kubernetes.io/zone", 1, LabelSelector({"app": "w"}),
                                                  "DoNotSchedule", None, None, "Honor")])
    res = _solve(request, backend, _problem(catalog, pools, [sh], [6]))
    assert sum(1 for p in res["placement"] if p != -1) >= 3


@pytest.mark.parametrize("backend", BACKENDS)
def test_relaxed_level_spread_group_with_ignore_policy(request, catalog, backend):
    """A DoNotSchedule zone spread with the DEFAULT taint policy (Ignore). Upstream MakeTopologyNodeFilter keeps the
    pod's tolerations under every policy and TopologyGroup.Hash hashes them, so the PreferNoSchedule level's group is a
    new group counted from the cluster alone (Topology.Update): the in-flight placement of the unrelaxed level is not in
    its counts. The untainted pool admits test-zone-1a only and one c5.xlarge (cpu limit): pod 2 fails its level (1a
    holds pod 1), relaxes, and the new group lets it join pod 1's NodeClaim in 1a; with the old group (in-flight counts
    kept) it would have gone to the tainted pool in another zone. Pods 3 and 4 then spread over 1b and 1c."""
    from kpamd import synth
    from kpamd.model import LabelSelector, PodShape, TopologySpread
    pools = _pools(plain_limit_cpu=4000, plain_zone="test-zone-1a")
    pools[0].requirements = [r for r in pools[0].requirements if r[0] != "topology.kubernetes.io/zone"]  # soft: all AZs
    sh = PodShape(synth.req_res(1000, 512), labels={"app": "w"},
                  topology_spread=[TopologySpread("topology.kubernetes.io/zone", 1, LabelSelector({"app": "w"}))])
    res = _solve(request, backend, _problem(catalog, pools, [sh], [4]))
    got = _pools_of(res, pools)
    assert got == ["plain", "plain", "soft", "soft"], got
    assert res["placement"][0] == res["placement"][1]
    zones = [dict((k, v) for k, op, v, *_ in n["requirements"] if op == "In").get("topology.kubernetes.io/zone")
             for n in res["nodeclaims"]]
    assert sorted(tuple(z) for z in zones) == [("test-zone-1a",), ("test-zone-1b",), ("test-zone-1c",)], zones


@pytest.mark.parametrize("backend", BACKENDS)
def test_compile_adds_the_level(request, catalog, backend):
    """The compile gives a shape one more relaxation level exactly when a NodePool carries a PreferNoSchedule taint and
    the shape lacks the exact toleration: a pod that fits nowhere is popped once per level (Relax re-queues it after
    each step), so its pops grow by one with the tainted pool, and not at all when it carries the toleration. The
    host compile (kp_solve_validate) accepts every variant."""
    import kpamd
    from kpamd import synth
    from kpamd.model import PodShape
    huge = synth.req_res(10_000_000, 512)  # fits no instance type
    shapes = {"plain": PodShape(dict(huge)), "tolerating": PodShape(dict(huge), tolerations=[("", "Exists", "", PNS)])}
    pops = {}
    for name, sh in shapes.items():
        for taint in (True, False):
            prob = _problem(catalog, _pools(soft_taint=taint), [sh], [1])
            assert kpamd.validate(prob) == 0
            res = _solve(request, backend, prob)
            assert list(res["placement"]) == [-1]
            pops[name, taint] = int(res["stats"]["pops"])
    assert pops["plain", True] == pops["plain", False] + 1, pops
    assert pops["tolerating", True] == pops["tolerating", False], pops


def _random(catalog, seed):
    from kpamd import synth
    return synth.random_problem(catalog, 1300 + seed, n_types=100, n_pods=260, n_pools=3, n_existing=10, n_shapes=16,
                                pns=0.5)


@pytest.mark.parametrize("seed", range(3))
def test_random_prefer_no_schedule_oracle_and_host_compile(catalog, seed):
    import kpamd
    from oracle import pyoracle
    prob = _random(catalog, seed)
    assert any(t[2] == PNS for p in prob.nodepools for t in p.taints)
    assert len(pyoracle.solve(prob)["placement"]) == prob.n_pods
    assert kpamd.validate(prob) == 0


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(8))
def test_gpu_random_prefer_no_schedule(ctx, catalog, seed):
    import kpamd
    from oracle import pyoracle
    from test_gpu_parity import check_same
    prob = _random(catalog, seed)
    check_same(kpamd.Scheduler(ctx, prob).solve(), pyoracle.solve(prob))


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(4))
def test_gpu_random_topology_prefer_no_schedule(ctx, catalog, seed):
    import kpamd
    from kpamd import synth
    from oracle import pyoracle
    from test_gpu_parity import check_same
    prob = synth.random_topology_problem(catalog, 1400 + seed, multi_terms=0.3, pns=0.5)
    check_same(kpamd.Scheduler(ctx, prob).solve(), pyoracle.solve(prob))


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(3))
def test_gpu_prefer_no_schedule_consolidation(ctx, catalog, seed):
    """Consolidation simulations relax the same way (the batched sim kernels index tolerations per shape-level)."""
    from kpamd import synth
    from test_gpu_consolidation import check
    cl = synth.random_cluster(catalog, 1500 + seed, n_nodes=30, pns=0.6)
    subs = synth.consolidation_subsets(cl, 16, seed=seed, max_size=10) + [[c] for c in cl.candidates[:8]]
    check(ctx, cl, subs, multi_node=bool(seed % 2))
