"""Host-side consolidation logic on CPU: the oracle's computeConsolidation on hand-built clusters (known
answers), the firstNConsolidationOption replay, subset generation, and the cross-rank best-decision
reduction over a world_size-2 gloo group."""
import os

import numpy as np
import pytest


def _mini_cluster(catalog, initialized_b=True, b_pods=1):
    """Node A: m5.large running one 500m pod; node B: m5.2xlarge with room. Both on-demand, zone 1a."""
    from kpamd import synth
    from kpamd.model import Cluster, ClusterNode, ExistingNode, NodePool, PodShape
    names = [it.name for it in catalog]
    shapes = [PodShape(synth.req_res(500, 512))]
    pool = NodePool("default", 0, 0, [("karpenter.sh/capacity-type", "In", ["on-demand"]),
                                      (synth.K + "instance-category", "In", ["c", "m", "r"])])
    nodes, pods = [], []
    for i, (tname, npods) in enumerate([("m5.large", 1), ("m5.2xlarge", b_pods)]):
        it = catalog[names.index(tname)]
        labels = synth.node_labels(it, 0, "on-demand", "default", f"n{i}")
        alloc = it.allocatable()
        mine = list(range(len(pods), len(pods) + npods))
        pods += [0] * npods
        used = {"cpu": 500 * npods, "memory": 512 * synth.MI * 1000 * npods, "pods": 1000 * npods}
        avail = {r: alloc[r] - used[r] for r in used}
        nodes.append(ClusterNode(ExistingNode(f"n{i}", labels, avail, {}, [], initialized_b or i == 0),
                                 0, names.index(tname), mine))
    n = len(pods)
    return Cluster([catalog], [pool], nodes, shapes, np.zeros(n, dtype=np.uint32),
                   np.full(n, 1_750_000_000, dtype=np.int64), np.arange(n, dtype=np.uint64), candidates=[0, 1])


def test_delete_when_pods_fit_elsewhere(catalog):
    from oracle import pyoracle
    cl = _mini_cluster(catalog)
    (r,), _ = pyoracle.simulate_batch(cl, [[0]], multi_node=False)
    assert r["decision"] == 1 and r["n_pods"] == 1
    assert r["savings"] == r["candidate_price"] > 0


def test_uninitialized_destination_is_noop(catalog):
    from oracle import pyoracle
    cl = _mini_cluster(catalog, initialized_b=False)
    (r,), _ = pyoracle.simulate_batch(cl, [[0]], multi_node=False)
    assert r["decision"] == 0


def test_replace_both_with_cheaper(catalog):
    """Both nodes' 2 pods (1 vCPU) fit one new NodeClaim cheaper than m5.large + m5.2xlarge."""
    from oracle import pyoracle
    cl = _mini_cluster(catalog)
    (r,), _ = pyoracle.simulate_batch(cl, [[0, 1]], multi_node=True)
    assert r["decision"] == 2 and r["n_pods"] == 2
    assert 0 < r["replacement_price"] < r["candidate_price"]
    assert r["savings"] == pytest.approx(r["candidate_price"] - r["replacement_price"])
    assert 1 <= r["n_options"] <= 100


def _with_pending(cl, requests):
    """Append one provisionable pod bound to no node (a new shape with these requests)."""
    from kpamd import synth
    from kpamd.model import PodShape
    cl.shapes = list(cl.shapes) + [PodShape(synth.req_res(*requests))]
    cl.pod_shape = np.append(cl.pod_shape, np.uint32(len(cl.shapes) - 1))
    cl.pod_creation = np.append(cl.pod_creation, np.int64(1_750_000_100))
    cl.pod_uid = np.append(cl.pod_uid, np.uint64(len(cl.pod_uid)))
    cl.pending = list(cl.pending) + [len(cl.pod_shape) - 1]
    return cl


def test_pending_pod_error_does_not_block(catalog):
    """A pending pod that fits nowhere joins the simulation, but only non-pending pods must schedule
    (AllNonPendingPodsScheduled): the delete stands, and the simulation counts both pods."""
    from oracle import pyoracle
    cl = _with_pending(_mini_cluster(catalog), (10_000_000, 64))
    (r,), _ = pyoracle.simulate_batch(cl, [[0]], multi_node=False)
    assert r["decision"] == 1 and r["n_pods"] == 2


def test_pending_pod_needing_a_nodeclaim(catalog):
    """A pending pod that needs a new NodeClaim makes the result carry one: no longer a delete."""
    from oracle import pyoracle
    cl = _mini_cluster(catalog)
    (r0,), _ = pyoracle.simulate_batch(cl, [[0]], multi_node=False)
    assert r0["decision"] == 1
    cl = _with_pending(cl, (7_000, 1024))  # larger than node B's room
    (r,), _ = pyoracle.simulate_batch(cl, [[0]], multi_node=False)
    assert r["decision"] != 1 and r["n_pods"] == 2


def test_deleting_node_pods_join(catalog):
    """A node marked for deletion is no destination and its pods reschedule in every simulation; a subset naming
    it is an error."""
    from oracle import pyoracle
    cl = _mini_cluster(catalog, b_pods=2)
    cl.nodes[1].deleting = True  # B: its two pods join, and A's pod has nowhere left but a new NodeClaim
    (r,), _ = pyoracle.simulate_batch(cl, [[0]], multi_node=False)
    assert r["n_pods"] == 3 and r["decision"] != 1
    with pytest.raises(RuntimeError):
        pyoracle.simulate_batch(cl, [[1]], multi_node=False)


def test_nodepool_limits_in_simulation(catalog):
    """kp_nodepool limits are the remaining limits: with no cpu left the replacement NodeClaim cannot be created."""
    from oracle import pyoracle
    cl = _mini_cluster(catalog)
    (r,), _ = pyoracle.simulate_batch(cl, [[0, 1]], multi_node=True)
    assert r["decision"] == 2
    cl.nodepools[0].limits = {"cpu": 0}
    (r,), _ = pyoracle.simulate_batch(cl, [[0, 1]], multi_node=True)
    assert r["decision"] == 0


def _spot_cluster(catalog):
    """One spot m5.2xlarge running one 500m pod and no other node: removing it needs a replacement; the pool
    allows spot and on-demand."""
    from kpamd import synth
    from kpamd.model import Cluster, ClusterNode, ExistingNode, NodePool, PodShape
    names = [it.name for it in catalog]
    shapes = [PodShape(synth.req_res(500, 512))]
    pool = NodePool("default", 0, 0, [("karpenter.sh/capacity-type", "In", ["on-demand", "spot"]),
                                      (synth.K + "instance-category", "In", ["c", "m", "r"])])
    it = catalog[names.index("m5.2xlarge")]
    labels = synth.node_labels(it, 0, "spot", "default", "n0")
    alloc = it.allocatable()
    avail = {r: alloc[r] - u for r, u in (("cpu", 500), ("memory", 512 * synth.MI * 1000), ("pods", 1000))}
    nodes = [ClusterNode(ExistingNode("n0", labels, avail, {}, [], True), 0, names.index("m5.2xlarge"), [0])]
    return Cluster([catalog], [pool], nodes, shapes, np.zeros(1, dtype=np.uint32),
                   np.full(1, 1_750_000_000, dtype=np.int64), np.arange(1, dtype=np.uint64), candidates=[0])


def test_spot_to_spot_gate(catalog):
    """All-spot candidates with a spot-capable replacement: no-op with the SpotToSpotConsolidation gate off;
    with it on, a replacement among >= 15 cheaper spot options, and the launch keeps 15 (disruption.md:110-128)."""
    from oracle import pyoracle
    cl = _spot_cluster(catalog)
    (r,), _ = pyoracle.simulate_batch(cl, [[0]], multi_node=False)
    assert r["decision"] == 0
    cl.spot_to_spot = True
    (r,), _ = pyoracle.simulate_batch(cl, [[0]], multi_node=False)
    assert r["decision"] == 2 and r["n_options"] == 15 and 0 < r["replacement_price"] < r["candidate_price"]


def test_first_n_replay():
    from kpamd.disruption import DELETE, NOOP, REPLACE, MultiNodeConsolidation as M
    n = 40
    # prefixes up to length 13 (mid 12) succeed, longer fail -> the search settles on mid 12
    by_mid = {m: {"decision": DELETE if m <= 12 else NOOP, "n_options": 0} for m in M.search_prefixes(n)}
    mid, r = M.replay(n, by_mid)
    assert mid == 12 and r["decision"] == DELETE
    by_mid = {m: {"decision": REPLACE, "n_options": 0} for m in M.search_prefixes(n)}  # no options left
    assert M.replay(n, by_mid) is None
    assert M.search_prefixes(1) == [] and M.search_prefixes(300)[-1] == 100  # prefix of 101 candidates
    assert M.search_prefixes(100)[-1] == 99 and M.search_prefixes(101)[-1] == 100 and M.search_prefixes(2) == [1]


def test_random_subsets_csr():
    from kpamd.disruption import random_subsets_csr
    offs, pos = random_subsets_csr(500, 1000, seed=3)
    assert offs[0] == 0 and len(offs) == 1001 and offs[-1] == len(pos)
    for i in range(1000):
        s = pos[offs[i]:offs[i + 1]]
        assert 1 <= len(s) <= 100 and np.all(np.diff(s.astype(np.int64)) > 0) and s.max() < 500


def _worker(rank, world, port, q):
    import torch.distributed as dist
    from kpamd.disruption import reduce_best, shard
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # rank 0 holds savings 3.0 at subset 7, rank 1 holds 3.0 at subset 5 and its shard is [50, 100)
        lo, hi = shard(100, rank, world)
        s, i = (3.0, 7) if rank == 0 else (3.0, 5)
        tie = reduce_best(s, i, dist, device="cpu")
        # strict winner on rank 0 at a higher index; rank 1 without any decision
        s, i = (4.5, 70) if rank == 0 else (-np.inf, -1)
        win = reduce_best(s, i, dist, device="cpu")
        none = reduce_best(-np.inf, -1, dist, device="cpu")
        q.put((rank, (lo, hi), tie, win, none))
    finally:
        dist.destroy_process_group()


def test_reduce_best_gloo_world2():
    import multiprocessing as mp
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    out = [q.get(timeout=120) for _ in ps]
    for p in ps:
        p.join(timeout=60)
    out.sort()
    assert out[0][1] == (0, 50) and out[1][1] == (50, 100)
    assert out[0][2] == out[1][2] == (3.0, 5)  # tie on savings -> lowest subset index
    assert out[0][3] == out[1][3] == (4.5, 70)
    assert out[0][4] == out[1][4] == (-np.inf, -1)


def _sweep_worker(rank, world, port, q):
    """One rank of the sweep on the CPU-validated path: the oracle simulates this rank's contiguous share of the
    subsets, the rank's kp_choice record goes through a gloo all-gather, and libkp's kp_choice_reduce picks the
    best (the host step of kp_consolidate_argmin)."""
    import torch.distributed as dist
    import kpamd
    from kpamd import abi, catalog, disruption, synth
    from oracle import pyoracle
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        cat = catalog.build_catalog(kpamd.load_lib())
        cl = synth.config4(cat, n_nodes=80, seed=44)
        subs = synth.consolidation_subsets(cl, 40, seed=7, max_size=30)
        lo, hi = disruption.shard(len(subs), rank, world)
        res, _ = pyoracle.simulate_batch(cl, subs[lo:hi]) if hi > lo else ([], None)
        rec = disruption.local_choice(res, base_index=lo)
        raw = bytes(memoryview(rec))
        gathered = [None] * world
        dist.all_gather_object(gathered, raw)
        recs = [abi.Choice.from_buffer_copy(g) for g in gathered]
        best = kpamd.choice_reduce(recs)
        q.put((rank, kpamd.choice_dict(best)))
    finally:
        dist.destroy_process_group()


def test_sweep_argmin_gloo_world2():
    """World-size 2 sweep (gloo): each rank simulates real subsets of a config-4 cluster; the reduced best over the
    ranks equals the N=1 best over all subsets (savings desc, lowest global index), counts summed."""
    import multiprocessing as mp
    import socket
    import kpamd
    from kpamd import catalog, disruption, synth
    from oracle import pyoracle
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_sweep_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    out = dict(q.get(timeout=300) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    cat = catalog.build_catalog(kpamd.load_lib())
    cl = synth.config4(cat, n_nodes=80, seed=44)
    subs = synth.consolidation_subsets(cl, 40, seed=7, max_size=30)
    res, _ = pyoracle.simulate_batch(cl, subs)
    want = kpamd.choice_dict(kpamd.choice_reduce([disruption.local_choice(res, 0)]))
    assert out[0] == out[1] == want
    assert want["subset"] >= 0 and sum(want["counts"]) == len(subs)
