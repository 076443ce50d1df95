"""Batched consolidation simulations on the device (kp_cluster_simulate) vs the CPU oracle's
computeConsolidation (oracle/oracle.cpp kpo_simulate_batch) — decision, replacement NodePool, prices,
savings and option count must be identical for every subset."""
import pytest

pytestmark = pytest.mark.gpu

FIELDS = ("decision", "nodepool", "candidate_price", "replacement_price", "savings", "n_options", "n_pods")


def check(ctx, cluster, subsets, multi_node=True):
    import kpamd
    from oracle import pyoracle
    plan = kpamd.ClusterPlan(ctx, cluster)
    try:
        got, _ = plan.simulate(subsets, multi_node=multi_node)
    finally:
        plan.close()
    want, _ = pyoracle.simulate_batch(cluster, subsets, multi_node=multi_node)
    bad = [i for i, (g, w) in enumerate(zip(got, want)) if tuple(g[f] for f in FIELDS) != tuple(w[f] for f in FIELDS)]
    assert not bad, f"{len(bad)}/{len(subsets)} subsets differ; first {bad[0]}: device {got[bad[0]]} oracle {want[bad[0]]}"
    return got


def test_config4_small(ctx, catalog):
    from kpamd import synth
    cl = synth.config4(catalog, n_nodes=120, seed=4)
    got = check(ctx, cl, synth.consolidation_subsets(cl, 30, seed=5))
    kinds = {r["decision"] for r in got}
    assert {0, 1}.issubset(kinds)


def test_config4_single_node(ctx, catalog):
    from kpamd import synth
    cl = synth.config4(catalog, n_nodes=80, seed=9)
    check(ctx, cl, [[c] for c in cl.candidates], multi_node=False)


@pytest.mark.parametrize("seed", range(8))
def test_random_clusters(ctx, catalog, seed):
    from kpamd import synth
    cl = synth.random_cluster(catalog, seed, n_nodes=[20, 40, 70][seed % 3])
    subs = synth.consolidation_subsets(cl, 25, seed=seed, max_size=min(30, len(cl.nodes)))
    subs += [[c] for c in cl.candidates[:15]]
    check(ctx, cl, subs, multi_node=bool(seed % 2))


def test_repeat_and_empty(ctx, catalog):
    import kpamd
    from kpamd import synth
    cl = synth.config4(catalog, n_nodes=60, seed=3)
    subs = synth.consolidation_subsets(cl, 10, seed=1)
    plan = kpamd.ClusterPlan(ctx, cl)
    try:
        a, _ = plan.simulate(subs)
        b, _ = plan.simulate(subs[::-1])
        assert a == b[::-1]
        c, _ = plan.simulate([])
        assert c == []
    finally:
        plan.close()
