"""Cancellation of a running Solve (ABI v11 kp_cancel): upstream `Scheduler.Solve(ctx, pods)` observes ctx.Done()
between pods (SURVEY §5 failure handling, §8b `Solve(ctx, pods) (Results, error)`); the cgo shim sets the token when
ctx.Done() fires and returns ctx.Err(). solve_kernel polls the host-mapped flag about every 1,024
Queue pops, in the fast lane and on the full path; a cancelled run returns KP_E_CANCELED and leaves the plan usable."""
import threading
import time

import pytest


def test_cancel_symbols_exported(lib):
    for n in ("kp_cancel_create", "kp_cancel_set", "kp_cancel_reset", "kp_cancel_destroy", "kp_solve_run_cancellable",
              "kp_solve_cancellable"):
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
