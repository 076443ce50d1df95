"""Cancellation of a running Solve (ABI v11 kp_cancel): upstream `Scheduler.Solve(ctx, pods)` observes ctx.Done()
between pods (SURVEY §5 failure handling, §8b `Solve(ctx, pods) (Results, error)`); the cgo shim sets the token when
ctx.Done() fires and returns ctx.Err(). solve_kernel polls the host-mapped flag about every 1,024
Queue pops, in the fast lane and on the full path; a cancelled run returns KP_E_CANCELED and leaves the plan usable.

Consolidation (ABI v12): upstream runs each consolidation pass under a timeout and counts the expired ones
(karpenter_voluntary_disruption_consolidation_timeouts_total, R:website/content/en/preview/reference/metrics.md:186-187);
kp_cluster_simulate_cancellable / kp_consolidate_argmin_cancellable take the same token: sim_kernel reads it between a
wave's subsets, the general path before each launch and inside every simulation's Solve."""
import threading
import time

import pytest


def test_cancel_symbols_exported(lib):
    for n in ("kp_cancel_create", "kp_cancel_set", "kp_cancel_reset", "kp_cancel_destroy", "kp_solve_run_cancellable",
              "kp_solve_cancellable", "kp_cluster_simulate_cancellable", "kp_consolidate_argmin_cancellable"):
        assert hasattr(lib, n), n
    from kpamd import abi
    assert abi.KP_E_CANCELED == -6


@pytest.mark.gpu
def test_cancel_before_and_after(ctx, catalog):
    import kpamd
    from kpamd import abi, synth
    prob = synth.config1(catalog)
    plan = kpamd.Scheduler(ctx, prob).prepare()
    want = plan.run()
    tok = kpamd.Cancel(ctx)
    got = plan.run(cancel=tok)  # not set: an ordinary run
    assert list(got["placement"]) == list(want["placement"])
    tok.set()
    with pytest.raises(kpamd.KPError) as e:
        plan.run(cancel=tok)
    assert e.value.code == abi.KP_E_CANCELED
    tok.reset()
    got = plan.run(cancel=tok)
    assert list(got["placement"]) == list(want["placement"])
    tok.close()
    plan.close()


@pytest.mark.gpu
def test_cancel_during_a_long_solve(ctx, catalog):
    """A 100k-pod config-5 Solve (~1 s of kernel) cancelled 50 ms in stops within a few ms and returns
    KP_E_CANCELED; the same plan then runs to the same result as before."""
    import kpamd
    from kpamd import abi, synth
    prob = synth.config5(catalog, n_pods=100_000)
    plan = kpamd.Scheduler(ctx, prob).prepare()
    t0 = time.perf_counter()
    want = plan.run()
    full_s = time.perf_counter() - t0
    tok = kpamd.Cancel(ctx)
    err = {}

    def run():
        try:
            plan.run(cancel=tok)
        except kpamd.KPError as e:
            err["code"] = e.code
    th = threading.Thread(target=run)
    t0 = time.perf_counter()
    th.start()
    time.sleep(min(0.05, full_s / 4))
    tok.set()
    th.join(60)
    cancelled_s = time.perf_counter() - t0
    assert err.get("code") == abi.KP_E_CANCELED
    assert cancelled_s < full_s * 0.6, (cancelled_s, full_s)
    tok.reset()
    got = plan.run(cancel=tok)
    assert list(got["placement"]) == list(want["placement"])
    tok.close()
    plan.close()


def _cancel_midway(fn, tok, full_s):
    """Run fn() on a thread, set tok after ~a quarter of its uncancelled time; returns (error code, seconds)."""
    import kpamd
    err = {}

    def run():
        try:
            fn()
        except kpamd.KPError as e:
            err["code"] = e.code
    th = threading.Thread(target=run)
    t0 = time.perf_counter()
    th.start()
    time.sleep(min(0.1, full_s / 4))
    tok.set()
    th.join(120)
    assert not th.is_alive()
    return err.get("code"), time.perf_counter() - t0


@pytest.mark.gpu
@pytest.mark.parametrize("path", ["sweep", "general"])
def test_cancel_consolidation(ctx, catalog, path):
    """A consolidation batch (the batched sim_kernel sweep on config 4, or the general path's batched Solves on the
    zone-spread cluster) cancelled before it starts and mid-run returns KP_E_CANCELED, well before the uncancelled
    time; the plan then gives the same choice as before (kp_consolidate_argmin) and the same per-subset results."""
    import numpy as np
    import kpamd
    from kpamd import abi, disruption, synth
    if path == "sweep":
        cl = synth.config4(catalog, n_nodes=2000, seed=4)
        offs, nodes, _ = disruption.sweep_subsets(np.asarray(cl.candidates, dtype=np.uint32), 400_000)
    else:
        cl = synth.spread_cluster(catalog, 2000)
        subs = synth.consolidation_subsets(cl, 24_000, seed=6, max_size=60, prefixes=False)
        offs = np.zeros(len(subs) + 1, dtype=np.uint32)
        offs[1:] = np.cumsum([len(x) for x in subs])
        nodes = np.concatenate([np.asarray(x, dtype=np.uint32) for x in subs])
    plan = kpamd.ClusterPlan(ctx, cl)
    tok = kpamd.Cancel(ctx)
    try:
        plan.argmin(offs[:9], nodes)  # warm (the general path builds its superset Solve on first use)
        t0 = time.perf_counter()
        want, want_res, _ = plan.argmin(offs, nodes, read_all=True, cancel=tok)  # token not set: an ordinary run
        full_s = time.perf_counter() - t0
        tok.set()
        with pytest.raises(kpamd.KPError) as e:
            plan.argmin(offs, nodes, cancel=tok)
        assert e.value.code == abi.KP_E_CANCELED
        with pytest.raises(kpamd.KPError) as e:
            plan.simulate_csr(offs[:9], nodes, cancel=tok)
        assert e.value.code == abi.KP_E_CANCELED
        tok.reset()
        code, s = _cancel_midway(lambda: plan.argmin(offs, nodes, cancel=tok), tok, full_s)
        assert code == abi.KP_E_CANCELED, code
        assert s < 0.6 * full_s + 0.05, (s, full_s)
        tok.reset()
        got, got_res, _ = plan.argmin(offs, nodes, read_all=True, cancel=tok)
        assert got == want
        assert (got_res == want_res).all()
    finally:
        tok.close()
        plan.close()
