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
