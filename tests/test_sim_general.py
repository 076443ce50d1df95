"""Consolidation simulations the batched sim kernels do not model, run as whole Solves on the device (the general
path of kp_cluster_prepare / kp_cluster_simulate / kp_consolidate_argmin): topology spread (counts seeded by every
pod still bound to a remaining node, Topology.countDomains skipping the pods being scheduled) and a pod
NotIn/DoesNotExist requirement on a label key some node lacks. Device decisions must equal the CPU oracle's
computeConsolidation (oracle/oracle.cpp kpo_simulate_batch) subset by subset; docs
R:website/content/en/preview/concepts/disruption.md:89-128. Parity unpinned beyond the written semantics (upstream
SimulateScheduling is not in the container)."""
import copy
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def cluster_with_spread(catalog, seed, n_nodes=30):
    from kpamd import synth
    from kpamd.model import LabelSelector, TopologySpread
    cl = synth.random_cluster(catalog, seed, n_nodes=n_nodes)
    rng = np.random.default_rng(seed)
    for i, sh in enumerate(cl.shapes):
        sh.labels = {"app": f"app-{i % 5}"}
        if rng.random() < 0.5 and len(sh.required_terms) <= 1:
            key = str(rng.choice(["topology.kubernetes.io/zone", "kubernetes.io/hostname"]))
            sh.topology_spread = [TopologySpread(key, int(rng.integers(1, 4)),
                                                 LabelSelector({"app": f"app-{i % 5}"}),
                                                 "DoNotSchedule" if rng.random() < 0.7 else "ScheduleAnyway")]
    return cl


def cluster_with_missing_key(catalog, seed):
    from kpamd import synth
    cl = synth.random_cluster(catalog, seed, n_nodes=30)
    for n in cl.nodes[::3]:
        n.node.labels = dict(n.node.labels, team="blue")
    cl.shapes[0].required_terms = [[("team", "NotIn", ["red"])]]
    cl.shapes[1].required_terms = [[("team", "DoesNotExist", [])]]
    return cl


def subsets_of(cl, seed):
    from kpamd import synth
    subs = synth.consolidation_subsets(cl, 15, seed=seed, max_size=min(12, len(cl.nodes)))
    return subs + [[c] for c in cl.candidates[:10]]


@pytest.mark.parametrize("seed", range(3))
def test_oracle_spread_simulations(catalog, seed):
    from oracle import pyoracle
    cl = cluster_with_spread(catalog, seed)
    subs = subsets_of(cl, seed)
    res, _ = pyoracle.simulate_batch(cl, subs)
    assert len(res) == len(subs)
    assert {r["decision"] for r in res} & {1, 2}, "some subset should delete or replace"


def test_product_host_compile_accepts_spread_clusters(catalog):
    """The general path's validation compile (every node existing, every pod pending) accepts the clusters."""
    import kpamd
    from kpamd.model import Problem
    for cl in (cluster_with_spread(catalog, 1), cluster_with_missing_key(catalog, 2)):
        prob = Problem(cl.catalogs, cl.nodepools, cl.shapes, cl.pod_shape, cl.pod_creation, cl.pod_uid,
                       existing=[n.node for n in cl.nodes])
        assert kpamd.validate(prob) == 0


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(6))
def test_gpu_spread_simulations(ctx, catalog, seed, general_mode):
    from test_gpu_consolidation import check
    cl = cluster_with_spread(catalog, 40 + seed, n_nodes=[20, 30, 40][seed % 3])
    check(ctx, cl, subsets_of(cl, seed), multi_node=bool(seed % 2))


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(2))
def test_gpu_missing_key_simulations(ctx, catalog, seed, general_mode):
    from test_gpu_consolidation import check
    cl = cluster_with_missing_key(catalog, 60 + seed)
    check(ctx, cl, subsets_of(cl, seed), multi_node=bool(seed % 2))


@pytest.mark.gpu
def test_gpu_spread_argmin_and_disruption(ctx, catalog, general_mode):
    """kp_consolidate_argmin over the general path (device argmax of host-taken decisions), and the
    firstNConsolidationOption replay in kpamd.disruption on a topology cluster, against the oracle."""
    import kpamd
    from kpamd import disruption
    from oracle import pyoracle
    cl = cluster_with_spread(catalog, 7, n_nodes=40)
    subs = subsets_of(cl, 7)
    plan = kpamd.ClusterPlan(ctx, cl)
    try:
        got, _ = plan.simulate(subs)
        want, _ = pyoracle.simulate_batch(cl, subs)
        assert [(g["decision"], g["savings"]) for g in got] == [(w["decision"], w["savings"]) for w in want]
        offs = np.zeros(len(subs) + 1, np.uint32)
        offs[1:] = np.cumsum([len(x) for x in subs])
        flat = np.concatenate([np.asarray(x, np.uint32) for x in subs])
        best, per, _ = plan.argmin(offs, flat, read_all=True)
        assert [int(x) for x in per["decision"]] == [w["decision"] for w in want]
        cands = [i for i, w in enumerate(want) if w["decision"] != 0]
        if cands:
            top = max(want[i]["savings"] for i in cands)
            assert best["subset"] == min(i for i in cands if want[i]["savings"] == top)
        else:
            assert best["subset"] == -1
    finally:
        plan.close()


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(4))
def test_gpu_batched_simulations_counted(ctx, catalog, seed, ov):
    """Every subset of a spread cluster runs batched (the superset Solve), and the decisions equal the per-subset
    compile's subset by subset (the oracle too): batched == single == oracle, savings included."""
    import kpamd
    from oracle import pyoracle
    cl = cluster_with_spread(catalog, 90 + seed, n_nodes=[16, 24, 36, 48][seed])
    subs = subsets_of(cl, seed) + [list(cl.candidates[:k]) for k in (2, 5, 9) if k <= len(cl.candidates)]
    runs = {}
    for mode in ("1", "0"):
        ov(general_batch=0 if mode == "1" else 1)
        plan = kpamd.ClusterPlan(ctx, cl)
        try:
            runs[mode] = plan.simulate(subs, multi_node=bool(seed % 2))
        finally:
            plan.close()
    (b, bst), (s, sst) = runs["1"], runs["0"]
    assert bst["phase_cycles"][:2] == [len(subs), 0] and sst["phase_cycles"][:2] == [0, len(subs)]
    want, _ = pyoracle.simulate_batch(cl, subs, multi_node=bool(seed % 2))
    for i, (x, y, w) in enumerate(zip(b, s, want)):
        assert x == y, (i, x, y)
        assert (x["decision"], x["savings"]) == (w["decision"], w["savings"]), (i, x, w)


@pytest.mark.gpu
@pytest.mark.parametrize("bad,msg", [("twice", "twice"), ("range", "node 9999"), ("order", "not monotone")])
def test_general_invalid_subsets(ctx, catalog, bad, msg):
    """A bad subset in a general-path batch (checked on the host threads): KP_E_INVAL naming the first bad subset, as
    the serial check reports it; the plan stays usable afterwards."""
    import numpy as np
    import kpamd
    from kpamd import synth
    cl = synth.spread_cluster(catalog, 40)
    cands = [int(c) for c in cl.candidates]
    subs = [cands[i:i + 3] for i in range(0, 30, 3)]
    if bad == "twice":
        subs[6] = [cands[0], cands[1], cands[0]]
        subs[8] = [cands[2], cands[2]]
    elif bad == "range":
        subs[4] = [cands[0], 9999]
        subs[7] = [9998]
    offs = np.zeros(len(subs) + 1, dtype=np.uint32)
    offs[1:] = np.cumsum([len(x) for x in subs])
    flat = np.concatenate([np.asarray(x, dtype=np.uint32) for x in subs])
    if bad == "order":
        offs[5] = offs[6] + 1
    plan = kpamd.ClusterPlan(ctx, cl)
    try:
        with pytest.raises(kpamd.KPError) as e:
            plan.simulate_csr(offs, flat)
        assert e.value.code == kpamd.abi.KP_E_INVAL
        want = {"twice": "subset 6", "range": "subset 4", "order": "at 5"}[bad]
        assert msg in str(e.value) and want in str(e.value), str(e.value)
        good = [cands[i:i + 3] for i in range(0, 9, 3)]
        res, _ = plan.simulate(good)
        assert len(res) == 3
    finally:
        plan.close()
