"""One bench leg alone, for rocprofv3 passes whose counters must belong to ONE kernel variant (tools/pmc_traffic.py
keys its figures by the leg this program ran, not by kernel name + grid size: the price-row and compact feasibility
launches are the same feasibility_quad_kernel at the same grid).

usage: prof_leg.py <leg> [reps]
  solve2         config 2 Solve (50k pods): one cold Solve, then `reps` Solves           -> solve_kernel<4,false,false>
  feas_rows      CompatibleAvailableFilter with the cheapest-price rows, 50k distinct rows -> feasibility_quad_kernel
  feas_compact   the same rows, compact result (mask + offering classes)                 -> feasibility_quad_kernel
  sweep          config 4: 1M random subsets of a 10k-node cluster, ONE kp_consolidate_argmin launch -> sim_kernel
  general        the 10k-node zone-spread cluster: 100 firstN prefixes + 8,092 random subsets (two launches of
                 4,096 simulations)                                                      -> solve_kernel<4,true,true>
Prints one JSON line: the leg's algorithmic bytes and device time per launch as the bench computes them."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "karpenter-provider-aws_amd"))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402

import kpamd  # noqa: E402
from kpamd import catalog, disruption, synth  # noqa: E402

ROW_BYTES = 880 + 96


def main():
    leg = sys.argv[1]
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    lib = kpamd.load_lib()
    cat = catalog.build_catalog(lib)
    ctx = kpamd.Context(0)
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import _ov  # (tools only: KP_HOST_TIMING=1 etc. -> kp_overrides)
    _ov.apply(ctx)
    out = {"leg": leg}
    if leg == "solve2":
        sched = kpamd.Scheduler(ctx, synth.config2(cat, n_pods=50_000, seed=2))
        sched.solve(read=False)
        st = [sched.solve(read=False)["stats"] for _ in range(reps)]
        out.update(launches=reps, kernel_ms=sum(s["solve_kernel_ms"] for s in st) / reps,
                   bytes_algorithmic=sum(s["bytes_algorithmic"] for s in st) / reps)
    elif leg in ("feas_rows", "feas_compact"):
        ch = kpamd.Catalog(ctx, cat)
        qs = synth.distinct_queries(cat, 50_000)
        T = len(cat)
        if leg == "feas_rows":
            fp = kpamd.FilterPlan(ctx, ch, qs, cheapest=True)
            fp.run()  # (warm)
            st = [fp.run() for _ in range(reps)]
            alg = len(qs) * (ROW_BYTES + 8 * T + 8 * ((T + 63) // 64))
        else:
            fp = kpamd.FilterPlan(ctx, ch, qs, cheapest="compact")
            fp.run_compact(read=False)  # (warm)
            st = [fp.run_compact(read=False) for _ in range(reps)]
            alg = len(qs) * (ROW_BYTES + 8 * ((T + 63) // 64) + 8)
        fp.close()
        ch.close()
        out.update(launches=reps, kernel_ms=sum(s["device_ms"] for s in st) / reps, bytes_algorithmic=alg)
    elif leg == "sweep":
        cl = synth.config4(cat, n_nodes=10_000, seed=4)
        offs, nodes, base = disruption.sweep_subsets(np.asarray(cl.candidates, dtype=np.uint32), 1_000_000)
        plan = kpamd.ClusterPlan(ctx, cl)
        t0 = time.perf_counter()
        ch, _, st = plan.argmin(offs, nodes, base_index=base)
        out.update(launches=1, subsets=len(offs) - 1, kernel_ms=st["solve_kernel_ms"],
                   bytes_algorithmic=st["bytes_algorithmic"], wall_s=time.perf_counter() - t0,
                   counts=ch["counts"])
        plan.close()
    elif leg == "general":
        cl = synth.spread_cluster(cat, 10_000)
        cands = np.asarray(cl.candidates, dtype=np.uint32)
        mids = disruption.MultiNodeConsolidation.search_prefixes(len(cands))
        subs = [list(cands[:m + 1]) for m in mids]
        n_sub = int(os.environ.get("GEN_SUBSETS", "8192"))
        subs += synth.consolidation_subsets(cl, n_sub - len(mids), seed=6, max_size=100, prefixes=False)
        offs = np.zeros(len(subs) + 1, dtype=np.uint32)
        offs[1:] = np.cumsum([len(x) for x in subs])
        flat = np.concatenate([np.asarray(x, dtype=np.uint32) for x in subs])
        plan = kpamd.ClusterPlan(ctx, cl)
        ch, _, st = plan.argmin(offs, flat)
        plan.close()
        # totals over the launches (launch count and per-launch averages: the kernel trace / pmc_traffic.py)
        out.update(launches=None, subsets=len(subs), kernel_ms=st["solve_kernel_ms"],
                   bytes_algorithmic=st["bytes_algorithmic"], counts=ch["counts"], pops=st["pops"])
        if os.environ.get("KP_TIMING"):  # the batched Solves' phase split (solve_kernel probes, summed over sims)
            names = ["pop+stage", "existing", "sort", "inflight-commit", "templates", "record+bookkeeping",
                     "inflight-prepass", "inflight-attempts"]
            tot = sum(st["attempt_cycles"]) or 1
            out["phase_share"] = {k: round(v / tot, 4) for k, v in zip(names, st["attempt_cycles"])}
            out["cycles_per_sim"] = round(tot / len(subs), 1)
    else:
        raise SystemExit(f"unknown leg {leg}")
    ctx.close()
    out["achieved_GBs"] = out["bytes_algorithmic"] / (out["kernel_ms"] / 1e3) / 1e9
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
