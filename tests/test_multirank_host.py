"""Multi-rank collectives driven from ONE process (the Karpenter controller is a single leader-elected
process): one kp_ctx per rank, one OS thread per rank, a communicator per rank — kp_comm_init_all (RCCL,
distinct GPUs) or kp_comm_init_host (a host all-gather supplied by the caller; here an in-process thread
exchange, so two ranks can share the one GPU of a test box and run the real kernels).

CPU: the reduction refuses a failed rank's record, and the thread exchange itself.
GPU: the sweep's argmin over two ranks equals one rank over all subsets; a rank whose step fails (a bad subset)
makes every rank return an error instead of leaving its peer in the collective; the template-options table
row-sharded over two ranks (tmpl_feas_kernel on each rank's rows + the exchange) gives the Solve kp_solve gives;
ranks passing different batches fail together."""
import threading

import numpy as np
import pytest


def _run_ranks(fns, timeout=300):
    """Run fns[r]() on one thread each; returns the results (an exception is returned, not raised)."""
    out = [None] * len(fns)

    def go(r):
        try:
            out[r] = fns[r]()
        except Exception as e:  # noqa: BLE001 - the test inspects it
            out[r] = e
    ts = [threading.Thread(target=go, args=(r,)) for r in range(len(fns))]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout)
        assert not t.is_alive(), "a rank is still waiting in the collective"
    return out


def test_choice_reduce_refuses_failed_rank(lib):
    import kpamd
    from kpamd import abi
    ok = abi.Choice()
    ok.subset = 5
    ok.result.savings = 1.0
    bad = abi.Choice()
    bad.subset = abi.CHOICE_FAILED
    bad.counts[0] = 2**64 - 3  # KP_E_DEVICE as uint64
    with pytest.raises(kpamd.KPError) as e:
        kpamd.choice_reduce([ok, bad], lib)
    assert e.value.code == abi.KP_E_DEVICE
    assert kpamd.choice_dict(kpamd.choice_reduce([ok], lib))["subset"] == 5


def test_thread_allgather():
    import kpamd
    ag = kpamd.ThreadAllGather(3)
    res = _run_ranks([lambda r=r: [ag(r, bytes([r]) * 4) for _ in range(3)] for r in range(3)])
    want = [bytes([0]) * 4, bytes([1]) * 4, bytes([2]) * 4]
    assert all(x == [want] * 3 for x in res)


def _csr(subs):
    offs = np.zeros(len(subs) + 1, dtype=np.uint32)
    offs[1:] = np.cumsum([len(s) for s in subs])
    flat = np.concatenate([np.asarray(s, dtype=np.uint32) for s in subs]) if subs else np.zeros(0, np.uint32)
    return offs, flat


@pytest.fixture(scope="module")
def ctx2():
    import kpamd
    cs = [kpamd.Context(0), kpamd.Context(0)]
    yield cs
    for c in cs:
        c.close()


@pytest.mark.gpu
def test_argmin_two_ranks_one_process(ctx2, catalog):
    import kpamd
    from kpamd import synth
    cl = synth.config4(catalog, n_nodes=150, seed=4)
    subs = synth.consolidation_subsets(cl, 400, seed=6)
    n = len(subs)
    halves = [(0, n * 3 // 5), (n * 3 // 5, n)]
    ag = kpamd.ThreadAllGather(2)
    comms = [kpamd.Comm.host(ctx2[r], 2, r, ag) for r in range(2)]
    plans = [kpamd.ClusterPlan(ctx2[r], cl) for r in range(2)]
    try:
        def rank(r):
            lo, hi = halves[r]
            offs, flat = _csr(subs[lo:hi])
            return plans[r].argmin(offs, flat, base_index=lo, comm=comms[r])[0]
        got = _run_ranks([lambda r=r: rank(r) for r in range(2)])
        offs, flat = _csr(subs)
        one = plans[0].argmin(offs, flat)[0]
    finally:
        for p in plans:
            p.close()
        for c in comms:
            c.close()
    assert not any(isinstance(g, Exception) for g in got), got
    assert got[0] == got[1] == one
    assert sum(one["counts"]) == len(subs)


@pytest.mark.gpu
def test_argmin_failed_rank_fails_every_rank(ctx2, catalog):
    import kpamd
    from kpamd import synth
    cl = synth.config4(catalog, n_nodes=60, seed=3)
    subs = synth.consolidation_subsets(cl, 20, seed=1)
    ag = kpamd.ThreadAllGather(2)
    comms = [kpamd.Comm.host(ctx2[r], 2, r, ag) for r in range(2)]
    plans = [kpamd.ClusterPlan(ctx2[r], cl) for r in range(2)]
    try:
        def rank(r):
            s = subs if r == 0 else subs[:3] + [[10**6]]  # rank 1: a node index outside the cluster
            offs, flat = _csr(s)
            return plans[r].argmin(offs, flat, base_index=100 * r, comm=comms[r])[0]
        got = _run_ranks([lambda r=r: rank(r) for r in range(2)])
    finally:
        for p in plans:
            p.close()
        for c in comms:
            c.close()
    assert isinstance(got[0], kpamd.KPError) and got[0].code == kpamd.abi.KP_E_DEVICE, got[0]
    assert isinstance(got[1], kpamd.KPError) and got[1].code == kpamd.abi.KP_E_INVAL, got[1]


def _canon(res):
    return (res["placement"].tolist(),
            [(nc["nodepool"], tuple(nc["pods"]), tuple(nc["options"])) for nc in res["nodeclaims"]])


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", ["2", "5"])
def test_prepare_sharded_table_two_ranks(ctx2, catalog, cfg):
    import kpamd
    from kpamd import synth
    for c in ctx2:  # shard every table (read when the communicator is created)
        c.set_overrides(table_shard_min=1)
    prob = synth.config2(catalog, n_pods=3000, seed=2) if cfg == "2" else synth.config5(catalog, n_pods=4000)
    ag = kpamd.ThreadAllGather(2)
    comms = [kpamd.Comm.host(ctx2[r], 2, r, ag) for r in range(2)]
    try:
        def rank(r):
            plan = kpamd.Scheduler(ctx2[r], prob).prepare(comms[r])
            try:
                return plan.run(read=True)
            finally:
                plan.close()
        got = _run_ranks([lambda r=r: rank(r) for r in range(2)])
    finally:
        for c in comms:
            c.close()
    assert not any(isinstance(g, Exception) for g in got), got
    want = _canon(kpamd.Scheduler(ctx2[0], prob).solve())
    assert _canon(got[0]) == _canon(got[1]) == want


@pytest.mark.gpu
def test_prepare_mismatched_batches_fail_together(ctx2, catalog):
    import kpamd
    from kpamd import synth
    for c in ctx2:
        c.set_overrides(table_shard_min=1)
    probs = [synth.config5(catalog, n_pods=500), synth.config2(catalog, n_pods=500, seed=2)]
    ag = kpamd.ThreadAllGather(2)
    comms = [kpamd.Comm.host(ctx2[r], 2, r, ag) for r in range(2)]
    try:
        got = _run_ranks([lambda r=r: kpamd.Scheduler(ctx2[r], probs[r]).prepare(comms[r]) for r in range(2)])
    finally:
        for c in comms:
            c.close()
    for g in got:
        assert isinstance(g, kpamd.KPError) and g.code == kpamd.abi.KP_E_INVAL, g
