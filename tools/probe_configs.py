#!/usr/bin/env python3
"""Full-size device runs of BASELINE configs 3 (100k pods, topology spread, 5k existing nodes) and 5 (1M-pod
burst, 20 pools): prepare + repeated Solve timings, and size-independent result properties. JSON to stdout."""
import json
import sys
import time
from collections import Counter
import os

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "karpenter-provider-aws_amd"))
import kpamd  # noqa: E402
from kpamd import catalog, synth  # noqa: E402


def run(name, prob, ctx, reps=2):
    t0 = time.perf_counter()
    plan = kpamd.Scheduler(ctx, prob).prepare()
    prep = time.perf_counter() - t0
    runs = []
    for _ in range(reps):
        t0 = time.perf_counter()
        st = plan.run(read=False)["stats"]
        runs.append((time.perf_counter() - t0, st))
    res = plan.run(read=True)
    plan.close()
    wall, st = runs[-1]
    out = {"config": name, "pods": prob.n_pods, "prepare_s": round(prep, 3), "wall_s": round(wall, 4),
           "solve_kernel_ms": round(st["solve_kernel_ms"], 3), "finalize_ms": round(st["finalize_kernel_ms"], 3),
           "pods_per_s": round(prob.n_pods / wall, 1), "nodeclaims": len(res["nodeclaims"]),
           "placed_existing": int((res["placement"] <= -2).sum()), "errors": int((res["placement"] == -1).sum()),
           "pops": st["pops"], "attempts": st["attempts"], "bytes": st["bytes_algorithmic"]}
    return out, res


def config3_properties(prob, res):
    shape = prob.pod_shape
    bound = Counter((e, lbl["app"]) for _, lbl, e in prob.bound_pods)
    placed = Counter()
    for p, pl in enumerate(res["placement"]):
        if pl <= -2:
            placed[(int(-2 - pl), prob.shapes[shape[p]].labels["app"])] += 1
    bad_ex = sum(1 for k, n in placed.items() if n != 1 or bound[k] != 0)
    bad_nc = bad_zone = 0
    for nc in res["nodeclaims"]:
        apps = Counter(prob.shapes[shape[p]].labels["app"] for p in nc["pods"])
        bad_nc += max(apps.values()) > 1
        z = [v for k, op, v, _ in nc["requirements"] if k == "topology.kubernetes.io/zone" and op == "In"]
        bad_zone += not (z and len(z[0]) == 1)
    return {"hostname_violations_existing": bad_ex, "hostname_violations_nodeclaims": bad_nc,
            "nodeclaims_not_single_zone": bad_zone}


def main():
    which = sys.argv[1:] or ["3", "5"]
    lib = kpamd.load_lib()
    cat = catalog.build_catalog(lib)
    ctx = kpamd.Context(0)
    if "2" in which:
        out, res = run("config2", synth.config2(cat, n_pods=50_000, seed=2), ctx)
        print(json.dumps(out), flush=True)
    if "3" in which:
        t0 = time.perf_counter()
        prob = synth.config3(cat)
        gen = time.perf_counter() - t0
        out, res = run("config3", prob, ctx)
        out["gen_s"] = round(gen, 2)
        out.update(config3_properties(prob, res))
        print(json.dumps(out), flush=True)
    if "5" in which:
        n = int(os.environ.get("KP_C5_PODS", "1000000"))
        prob = synth.config5(cat, n_pods=n)
        out, res = run("config5", prob, ctx, reps=1)
        print(json.dumps(out), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
