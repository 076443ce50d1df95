"""Handle lifetimes at the C ABI: a context destroyed before its dependents (the order a garbage collector may
finalize a reference cycle in) leaves them destroyable, and nothing is freed twice."""
import gc

import pytest


@pytest.mark.gpu
def test_context_destroyed_before_dependents(lib, catalog):
    import kpamd
    from kpamd import synth
    small_problem = synth.config1(catalog)
    ctx = kpamd.Context(0)
    cat = kpamd.Catalog(ctx, catalog)
    fp = kpamd.FilterPlan(ctx, cat, synth.distinct_queries(catalog, 4), cheapest=True)
    fp.run()
    plan = kpamd.Scheduler(ctx, small_problem).prepare()
    plan.run()
    ctx.close()  # the context goes first
    out = plan.run()  # a plan holds its context: it still runs
    assert out["stats"]["pops"] > 0
    plan.close()
    fp.close()
    cat.close()


@pytest.mark.gpu
def test_cycle_collected_in_any_order(lib, catalog):
    import kpamd
    from kpamd import synth
    small_problem = synth.config1(catalog)
    for _ in range(3):
        ctx = kpamd.Context(0)
        cat = kpamd.Catalog(ctx, catalog)
        plan = kpamd.Scheduler(ctx, small_problem).prepare()
        ctx.cycle = [ctx, cat, plan]  # one garbage cycle holding all three
        del ctx, cat, plan
        gc.collect()


@pytest.mark.gpu
def test_filter_and_launch_plans_after_catalogue_destroyed(ctx, lib, catalog):
    """kp_filter_run / kp_filter_refresh / kp_launch_run / kp_launch_refresh on a plan whose catalogue was destroyed
    return KP_E_INVAL (the plan holds the catalogue's alive token) instead of reading freed memory."""
    import kpamd
    from kpamd import catalog as kc
    from kpamd import synth
    cat = kpamd.Catalog(ctx, catalog)
    fp = kpamd.FilterPlan(ctx, cat, synth.distinct_queries(catalog, 4), cheapest=True)
    lp = kpamd.LaunchPlan(ctx, cat, synth.random_launch_requests(catalog, 8, seed=5), kc.ZONES)
    fp.run(read=True)
    lp.run(read=True)
    cat2 = kpamd.Catalog(ctx, catalog)
    cat_h = cat.h
    cat.close()
    for call in (lambda: fp.run(read=True), lambda: lp.run(read=True)):
        with pytest.raises(kpamd.KPError, match="destroyed") as e:
            call()
        assert e.value.code == -1  # KP_E_INVAL
    for plan in (fp, lp):  # a refresh on the destroyed catalogue's handle, or on another one
        cat.h = cat_h
        with pytest.raises(kpamd.KPError, match="destroyed"):
            plan.refresh(cat)
        with pytest.raises(kpamd.KPError, match="destroyed"):
            plan.refresh(cat2)
    cat.h = None
    fp.close()
    lp.close()
    cat2.close()
