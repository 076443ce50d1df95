"""Topology spread on the device (solve_kernel with TopologyGroups) vs the CPU oracle — bit-exact placements,
NodeClaims, options and final requirements (zone narrowing included). SURVEY §8a a16, config 3."""
import pytest

from test_gpu_parity import check_same, run_both
import test_topology_oracle as kat

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("seed", range(16))
def test_random_topology(ctx, catalog, seed):
    from kpamd import synth
    prob = synth.random_topology_problem(catalog, seed, n_existing=[0, 12, 30][seed % 3])
    got, want = run_both(ctx, prob)
    check_same(got, want)


def test_config3_scaled(ctx, catalog):
    from kpamd import synth
    got, want = run_both(ctx, synth.config3(catalog, n_pods=3000, n_deployments=60, n_existing=150))
    check_same(got, want)


def test_topology_kats(ctx, catalog):
    from kpamd.model import ExistingNode
    from kpamd import synth
    probs = [
        kat.problem(catalog, [kat.spread_shape("a", kat.ZONE, cpu=3500)], [9]),
        kat.problem(catalog, [kat.spread_shape("a", kat.HOST, skew=3, cpu=100)], [7]),
        kat.problem(catalog, [kat.spread_shape("a", kat.ZONE, min_domains=4, cpu=100)], [5]),
        kat.problem(catalog, [kat.spread_shape("a", "example.com/rack"),
                              kat.spread_shape("b", "example.com/rack", when="ScheduleAnyway")], [3, 3]),
    ]
    it = catalog[synth._type_named(catalog, "m5.xlarge")]
    alloc = it.allocatable()
    nodes = [ExistingNode(f"n{z}", synth.node_labels(it, z, "on-demand", "default", f"n{z}"),
                          {k: alloc[k] for k in ("cpu", "memory", "pods")}) for z in range(3)]
    bound = [("default", {"app": "a"}, 0), ("default", {"app": "a"}, 0), ("other", {"app": "a"}, 1)]
    probs.append(kat.problem(catalog, [kat.spread_shape("a", kat.ZONE, cpu=100)], [4], existing=nodes, bound=bound))
    for prob in probs:
        got, want = run_both(ctx, prob)
        check_same(got, want)


@pytest.mark.parametrize("seed", range(12))
def test_random_topology_multi_terms(ctx, catalog, seed):
    """Spread pods with 2-3 required node-affinity terms: relaxation re-creates their groups (per-level groups, live
    from the first relaxation, hostname groups registering only later NodeClaims and countDomains' nodes)."""
    from kpamd import synth
    prob = synth.random_topology_problem(catalog, 100 + seed, n_existing=[0, 12, 30][seed % 3], multi_terms=0.5)
    got, want = run_both(ctx, prob)
    check_same(got, want)


def test_multi_term_kats(ctx, catalog):
    from kpamd import synth
    from kpamd.model import PodShape
    a = kat.spread_shape("a", kat.ZONE, cpu=3500)
    a.required_terms = [kat.CAT_X, kat.OD]
    b = kat.spread_shape("a", kat.ZONE, cpu=3600)
    c = PodShape(synth.req_res(500, 1024), labels={"app": "a"})
    h = kat.spread_shape("a", kat.HOST, cpu=400)
    h.required_terms = [kat.CAT_X, kat.OD]
    for prob in [kat.problem(catalog, [a], [9]), kat.problem(catalog, [b, a], [2, 3]), kat.problem(catalog, [c, h], [2, 2])]:
        got, want = run_both(ctx, prob)
        check_same(got, want)


@pytest.mark.parametrize("n_groups,n_existing", [(12, 0), (12, 9), (70, 0), (70, 9)])
def test_many_recorded_groups(ctx, catalog, n_groups, n_existing):
    """Every pod is counted by n_groups spread groups (one per shape: the same tier selector, its own maxSkew, zone
    or hostname key): more than the stage record's 8 recorded groups (their list read from memory) and, at 70, more
    than one 64-lane Topology.Record pass (record_node instead of the reads issued ahead of the commit stores), on
    NodeClaims and on existing nodes."""
    from kpamd import synth
    from kpamd.model import ExistingNode, LabelSelector, PodShape, TopologySpread
    sel = LabelSelector(match_labels={"tier": "web"})
    shapes = [PodShape(synth.req_res(100 + 50 * (i % 5), 256), labels={"app": f"d{i}", "tier": "web"},
                       topology_spread=[TopologySpread(kat.ZONE if i % 2 == 0 else kat.HOST, 2 + i, sel)])
              for i in range(n_groups)]
    it = catalog[synth._type_named(catalog, "m5.xlarge")]
    alloc = it.allocatable()
    nodes = [ExistingNode(f"n{e}", synth.node_labels(it, e % 3, "on-demand", "default", f"n{e}"),
                          {k: alloc[k] for k in ("cpu", "memory", "pods")}) for e in range(n_existing)]
    prob = kat.problem(catalog, shapes, [3] * n_groups, existing=nodes)
    got, want = run_both(ctx, prob)
    check_same(got, want)
