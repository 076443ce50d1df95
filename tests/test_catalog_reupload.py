"""A `List` cache miss without a seqnum change: `DefaultProvider.get` overrides `Capacity[memory]`
with the memory a launched node reported (`UpdateInstanceTypeCapacityFromNode`,
R:pkg/providers/instancetype/instancetype.go:213-215,330-355), and that value reaches `List`'s result when its
instance-type cache entry expires (`:145-160`) — no seqnum moves. The shim therefore re-uploads whenever `List` returns
a rebuilt slice (INTEGRATION.md `UploadCatalog`), and the new handle must never hit a SolveBase compiled from the old
one: the ctx cache keys bases by catalogue upload identity (a fresh uid per `kp_catalog_upload`), not by seqnum alone.

The test: one NodePool restricted to m5.large, a pod whose memory request is just above m5.large's allocatable memory
(pending), then the same catalogue with m5.large's memory capacity raised as a node's reported capacity would, uploaded
as a new handle with the SAME seqnum: the Solve must compile a new base (catalog_cached = 0) and place the pod, equal
to the oracle on the changed catalogue; the old handle keeps its resident base and its answer."""
import copy

import pytest

GI = 1 << 30


def _problem(cat, mem_milli):
    from kpamd.model import NodePool, PodShape, Problem
    import scenarios
    pool = NodePool("m5l", 0, 0, [("node.kubernetes.io/instance-type", "In", ["m5.large"]),
                                  ("karpenter.sh/capacity-type", "In", ["on-demand"])])
    s, c, u = scenarios.pods_of([2])
    return Problem([cat], [pool], [PodShape({"cpu": 500, "memory": mem_milli, "pods": 1000})], s, c, u, name="reupload")


def _changed(catalog, extra_mem_milli):
    cat = copy.deepcopy(catalog)
    it = next(t for t in cat if t.name == "m5.large")
    it.capacity = dict(it.capacity, memory=it.capacity["memory"] + extra_mem_milli)
    return cat


def test_changed_capacity_changes_the_oracle_answer(catalog):
    """(CPU) the scenario is live: pending on the listed capacity, placed on the discovered one."""
    from oracle import pyoracle
    it = next(t for t in catalog if t.name == "m5.large")
    mem = it.allocatable()["memory"] + 64 * (1 << 20) * 1000
    assert all(p == -1 for p in pyoracle.solve(_problem(catalog, mem))["placement"])
    assert all(p >= 0 for p in pyoracle.solve(_problem(_changed(catalog, GI * 1000), mem))["placement"])


@pytest.mark.gpu
def test_reupload_same_seqnum_is_not_a_cache_hit(ctx, catalog):
    import kpamd
    from oracle import pyoracle
    from test_gpu_parity import check_same
    it = next(t for t in catalog if t.name == "m5.large")
    mem = it.allocatable()["memory"] + 64 * (1 << 20) * 1000
    old_prob = _problem(catalog, mem)
    old = kpamd.Catalog(ctx, catalog, seqnum=7)
    r0 = kpamd.Scheduler(ctx, old_prob, catalogs=[old]).solve()
    r1 = kpamd.Scheduler(ctx, old_prob, catalogs=[old]).solve()
    assert r1["stats"]["catalog_cached"] == 1  # the same upload: resident
    check_same(r0, pyoracle.solve(old_prob))
    new_cat = _changed(catalog, GI * 1000)
    new_prob = _problem(new_cat, mem)
    new = kpamd.Catalog(ctx, new_cat, seqnum=7)  # a rebuilt List slice, seqnum unchanged
    r2 = kpamd.Scheduler(ctx, new_prob, catalogs=[new]).solve()
    assert r2["stats"]["catalog_cached"] == 0
    check_same(r2, pyoracle.solve(new_prob))
    assert all(p >= 0 for p in r2["placement"])
    r3 = kpamd.Scheduler(ctx, old_prob, catalogs=[old]).solve()  # the old handle still answers for the old slice
    check_same(r3, pyoracle.solve(old_prob))
    old.close()
    new.close()
