"""Batched consolidation simulations on the device (kp_cluster_simulate) vs the CPU oracle's
computeConsolidation (oracle/oracle.cpp kpo_simulate_batch) — decision, replacement NodePool, prices,
savings and option count must be identical for every subset."""
import os
import sys

import pytest
import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

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
    cl = synth.config4(catalog, n_nodes=120, seed=4, loose=0.05)
    got = check(ctx, cl, synth.consolidation_subsets(cl, 30, seed=5))
    kinds = {r["decision"] for r in got}
    assert {0, 1, 2}.issubset(kinds)


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


def test_known_answers(ctx, catalog):
    from test_consolidation_host import _mini_cluster
    got = check(ctx, _mini_cluster(catalog), [[0], [1], [0, 1]], multi_node=True)
    assert got[0]["decision"] == 1 and got[2]["decision"] == 2
    got = check(ctx, _mini_cluster(catalog, initialized_b=False), [[0]], multi_node=False)
    assert got[0]["decision"] == 0


def test_multi_and_single_node_commands(ctx, catalog):
    """firstNConsolidationOption / SingleNodeConsolidation driven by device batches agree with the same
    searches driven by the oracle."""
    import kpamd
    from kpamd import synth
    from kpamd.disruption import MultiNodeConsolidation, SingleNodeConsolidation
    from oracle import pyoracle
    cl = synth.config4(catalog, n_nodes=150, seed=12)
    plan = kpamd.ClusterPlan(ctx, cl)
    try:
        multi = MultiNodeConsolidation(plan).first_n_option(cl.candidates)
        single = SingleNodeConsolidation(plan).compute_command(cl.candidates)
    finally:
        plan.close()
    mids = MultiNodeConsolidation.search_prefixes(len(cl.candidates))
    want, _ = pyoracle.simulate_batch(cl, [cl.candidates[:m + 1] for m in mids], multi_node=True)
    hit = MultiNodeConsolidation.replay(len(cl.candidates), dict(zip(mids, want)))
    assert (multi is None and hit is None) or (multi[0] == hit[0] + 1 and multi[1] == hit[1])
    want1, _ = pyoracle.simulate_batch(cl, [[c] for c in cl.candidates], multi_node=False)
    first = next(((c, r) for c, r in zip(cl.candidates, want1) if r["decision"] != 0), None)
    assert single == first


@pytest.mark.gpu
def test_consolidate_argmin_device(ctx, catalog):
    """kp_consolidate_argmin: the device argmax over a batch (+ the RCCL all-gather on a one-rank communicator)
    equals the host reduction of the per-subset results and of the oracle's (savings desc, lowest global index)."""
    import kpamd
    from kpamd import disruption, synth
    from oracle import pyoracle
    cl = synth.config4(catalog, n_nodes=120, seed=4)
    subs = synth.consolidation_subsets(cl, 300, seed=5)
    offs = np.zeros(len(subs) + 1, dtype=np.uint32)
    offs[1:] = np.cumsum([len(s) for s in subs])
    flat = np.concatenate([np.asarray(s, dtype=np.uint32) for s in subs])
    plan = kpamd.ClusterPlan(ctx, cl)
    comm = kpamd.Comm(ctx, kpamd.comm_unique_id(), 1, 0)
    try:
        ch, res, _ = plan.argmin(offs, flat, base_index=1000, read_all=True)
        ch2, _, _ = plan.argmin(offs, flat, base_index=1000, comm=comm)
        empty, _, _ = plan.argmin(np.zeros(1, dtype=np.uint32), np.zeros(0, dtype=np.uint32), base_index=7, comm=comm)
    finally:
        comm.close()
        plan.close()
    host = kpamd.choice_dict(kpamd.choice_reduce([disruption.local_choice(res, 1000)]))
    assert ch == ch2 == host
    want, _ = pyoracle.simulate_batch(cl, subs)
    oracle = kpamd.choice_dict(kpamd.choice_reduce([disruption.local_choice(want, 1000)]))
    assert ch == oracle
    assert empty["subset"] == -1 and empty["counts"] == [0, 0, 0]


@pytest.mark.parametrize("limit", [None, 16000, 4000])
def test_disruption_state_config4(ctx, catalog, limit):
    """Deleting nodes, pending pods (some unschedulable) and remaining NodePool limits (SimulateScheduling's
    other inputs) on a near-capacity config-4 cluster: device == oracle."""
    from kpamd import synth
    base = synth.config4(catalog, n_nodes=120, seed=4, loose=0.05)
    cl = synth.with_disruption_state(base, 7, cpu_limit_m=limit)
    subs = [[c for c in s if not cl.nodes[c].deleting] for s in synth.consolidation_subsets(base, 30, seed=5)]
    got = check(ctx, cl, [s for s in subs if s])
    assert {r["n_pods"] for r in got} != {0}


@pytest.mark.parametrize("seed", range(4))
def test_disruption_state_random(ctx, catalog, seed):
    from kpamd import synth
    base = synth.random_cluster(catalog, 100 + seed, n_nodes=40)
    cl = synth.with_disruption_state(base, seed, n_deleting=2, n_pending=4, cpu_limit_m=[None, 8000][seed % 2])
    subs = synth.consolidation_subsets(cl, 20, seed=seed, max_size=min(20, len(cl.candidates)))
    subs += [[c] for c in cl.candidates[:10]]
    check(ctx, cl, subs, multi_node=bool(seed % 2))


@pytest.mark.parametrize("seed", range(4))
def test_spot_to_spot_random(ctx, catalog, seed):
    """SpotToSpotConsolidation gate on: randomized clusters (30 % spot nodes), single- and multi-node, device ==
    oracle."""
    from kpamd import synth
    cl = synth.random_cluster(catalog, 200 + seed, n_nodes=40)
    cl.spot_to_spot = True
    spot = [c for c in cl.candidates if dict(cl.nodes[c].node.labels).get("karpenter.sh/capacity-type") == "spot"]
    subs = [[c] for c in spot[:15]] + [spot[i:i + 3] for i in range(0, max(0, len(spot) - 2), 2)]
    subs += synth.consolidation_subsets(cl, 10, seed=seed, max_size=min(10, len(cl.candidates)))
    check(ctx, cl, [s for s in subs if s], multi_node=bool(seed % 2))


@pytest.mark.parametrize("multi_node", [False, True])
def test_spot_to_spot_config4(ctx, catalog, multi_node):
    """Near-capacity config-4 cluster, gate on, spot-only candidate subsets (single nodes and triples): spot-to-spot
    replacements occur (15 options for a single node, all cheaper spot options for several) and device == oracle."""
    from kpamd import synth
    cl = synth.config4(catalog, n_nodes=200, seed=11)
    cl.spot_to_spot = True
    spot = [c for c in cl.candidates if dict(cl.nodes[c].node.labels).get("karpenter.sh/capacity-type") == "spot"]
    rng = np.random.default_rng(1)
    subs = [[c] for c in spot[:30]]
    subs += [sorted(rng.choice(spot, 3, replace=False).tolist(), key=cl.candidates.index) for _ in range(20)]
    got = check(ctx, cl, subs, multi_node=multi_node)
    repl = [r for r in got if r["decision"] == 2]
    assert repl and any(r["n_options"] == 15 for r in repl)

