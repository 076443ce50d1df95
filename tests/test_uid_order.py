"""NewQueue's last tie-break on the full UID string (ABI v10 kp_solve_in.pod_uids / kp_cluster.pod_uids).

Upstream NewQueue orders pods by cpu desc, memory desc, creationTimestamp asc, then UID asc (SURVEY a13 / Appendix B
item 1). A shim passing only an 8-byte UID prefix as kp_pod.uid_key would order pods sharing that prefix, creation
second and shape by batch index instead; with the UIDs themselves the library ranks them exactly. The batches here
give every pod its own NodeClaim (a 100-core request fits once on any type of the pool), so the NodeClaims' creation
order is the Queue order.
"""
import numpy as np
import pytest

from kpamd import synth
from kpamd.model import NodePool, PodShape, Problem

PREFIX = "7f3a9c21-"  # first 8 bytes shared by every UID (and creation second, and shape)


def _uids(rng, n):
    return [PREFIX + "%04x-%04x-%012x" % (rng.integers(0, 1 << 16), rng.integers(0, 1 << 16), rng.integers(0, 1 << 48))
            for _ in range(n)]


def _problem(catalog, n=12, seed=0, two_shapes=False):
    rng = np.random.default_rng(seed)
    shapes = [PodShape(synth.req_res(100_000, 1024))]
    if two_shapes:
        shapes.append(PodShape(synth.req_res(100_000, 2048)))  # more memory: ahead in the Queue
    shape = (np.arange(n) % len(shapes)).astype(np.uint32)
    creation = np.full(n, 1_750_000_000, dtype=np.int64)
    if two_shapes:
        creation[::3] -= 1  # an earlier creation second wins before the UID
    pool = NodePool("default", 0, 0, list(synth.KWOK_POOL_REQS))
    prob = Problem([catalog], [pool], shapes, shape, creation, np.zeros(n, dtype=np.uint64), name="uid-order")
    prob.pod_uid_str = _uids(rng, n)
    return prob


def _expected_order(prob):
    req = [(-s.requests["cpu"], -s.requests["memory"]) for s in prob.shapes]
    key = [(*req[int(prob.pod_shape[p])], int(prob.pod_creation[p]), prob.pod_uid_str[p]) for p in range(prob.n_pods)]
    return sorted(range(prob.n_pods), key=lambda p: key[p])


def _creation_order(res):
    assert all(len(n["pods"]) == 1 for n in res["nodeclaims"])
    return [n["pods"][0] for n in res["nodeclaims"]]


@pytest.mark.parametrize("seed,two", [(0, False), (1, True), (2, True)])
def test_oracle_orders_by_full_uid(catalog, seed, two):
    from oracle import pyoracle
    prob = _problem(catalog, seed=seed, two_shapes=two)
    want = _expected_order(prob)
    assert want != sorted(want), "the UIDs must disagree with the batch order for the test to mean anything"
    assert _creation_order(pyoracle.solve(prob)) == want


def test_validate_rejects_null_uid(lib, catalog):
    import ctypes as C

    from kpamd import abi
    prob = _problem(catalog)
    arena = abi.Arena()
    handles = []
    for c in prob.catalogs:
        h = C.c_void_p()
        a2 = abi.Arena()
        desc = a2.catalog_desc(c)
        assert lib.kp_catalog_upload(None, C.byref(desc), 1, C.byref(h)) == 0
        handles.append((h, a2))
    si = abi.build_solve_in(arena, prob, catalog_handles=[h.value for h, _ in handles])
    assert lib.kp_solve_validate(C.byref(si)) == 0
    si.pod_uids[3] = None
    assert lib.kp_solve_validate(C.byref(si)) == -1  # KP_E_INVAL
    for h, _ in handles:
        lib.kp_catalog_destroy(h)


@pytest.mark.gpu
@pytest.mark.parametrize("seed,two", [(0, False), (1, True), (3, True)])
def test_device_orders_by_full_uid(ctx, catalog, seed, two):
    import kpamd
    from oracle import pyoracle
    prob = _problem(catalog, n=40, seed=seed, two_shapes=two)
    got = kpamd.Scheduler(ctx, prob).solve()
    want = pyoracle.solve(prob)
    assert _creation_order(got) == _expected_order(prob) == _creation_order(want)
    assert (got["placement"] == want["placement"]).all()


@pytest.mark.gpu
def test_device_uid_strings_larger_batch(ctx, catalog):
    """config 2 with every UID sharing its first 8 bytes and creation second: device == oracle."""
    import kpamd
    from oracle import pyoracle
    from test_gpu_parity import check_same
    prob = synth.config2(catalog, n_pods=3000, seed=9)
    rng = np.random.default_rng(9)
    prob.pod_creation[:] = 1_750_000_000
    prob.pod_uid[:] = 0
    prob.pod_uid_str = _uids(rng, prob.n_pods)
    check_same(kpamd.Scheduler(ctx, prob).solve(), pyoracle.solve(prob))


@pytest.mark.gpu
@pytest.mark.parametrize("spread", [False, True])
def test_cluster_null_uid_is_invalid(ctx, catalog, general_mode, spread):
    """A NULL entry in kp_cluster.pod_uids is KP_E_INVAL on every consolidation path (batched kernels, the general
    path batched or per subset), as kp_solve rejects it — not a silent fallback to uid_key."""
    import kpamd
    from kpamd import synth
    cl = synth.spread_cluster(catalog, 40) if spread else synth.config4(catalog, n_nodes=40)
    rng = np.random.default_rng(3)
    uids = _uids(rng, len(cl.pod_shape))
    uids[len(uids) // 2] = None
    cl.pod_uid_str = uids
    with pytest.raises(kpamd.KPError) as e:
        kpamd.ClusterPlan(ctx, cl)
    assert e.value.code == kpamd.abi.KP_E_INVAL
