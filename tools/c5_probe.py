"""Config-5 probe: whole-Solve timing of the 1M-pod burst (or a prefix) on the device with the fast-lane and chunked
order counters. usage: c5_probe.py [pods] [limit_div]   (KP_TIMING=1 adds the phase split)"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "karpenter-provider-aws_amd"))
import kpamd  # noqa: E402
from kpamd import catalog, synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
div = int(sys.argv[2]) if len(sys.argv) > 2 else 1
lib = kpamd.load_lib()
cat = catalog.build_catalog(lib)
prob = synth.config5(cat, n_pods=n, limit_div=div)
ctx = kpamd.Context(0)
import _ov  # noqa: E402  (tools only: diagnostic variables -> kp_overrides)
_ov.apply(ctx)
plan = kpamd.Scheduler(ctx, prob).prepare()
out = {"pods": n, "limit_div": div, "runs": []}
for _ in range(int(os.environ.get("REPS", "2"))):
    t0 = time.perf_counter()
    st = plan.run(read=False)["stats"]
    wall = time.perf_counter() - t0
    out["runs"].append({"wall_s": round(wall, 3), "kernel_ms": round(st["solve_kernel_ms"], 1),
                        "pods_per_s": round(n / wall, 1)})
    print(json.dumps(out["runs"][-1]), file=sys.stderr, flush=True)
pops = max(1, st["pops"])
out.update({"pops": st["pops"], "attempts_per_pop": round(st["attempts"] / pops, 3), "fast_pods": st["fast_pods"],
            "fast_share": round(st["fast_pods"] / pops, 4), "scanned_per_pop": round(st["scanned"] / pops, 1),
            "cursor_start_per_pop": round(st["cursor_starts"] / pops, 1), "slow_sorts": st["slow_sorts"],
            "fast_bails": dict(zip(["ineligible", "spilled", "shift", "scan", "merge", "minvalues", "none", "memo"],
                                   st["fast_bails"])),
            "order_chunks": dict(zip(["peak_chunks", "splits", "emptied", "builds", "final_mode"], st["order_chunks"]))})
if os.environ.get("FX_DIAG"):  # variant build (tools/kp_diag.h FX_DIAG): the fast lane's memo pops
    out["memo_pops"] = dict(zip(["single", "batched", "single_after_placement", "batches"], st["fast_cycles"][:4]))
    out["new_nodeclaims"] = {"template_rounds": st["fast_cycles"][4], "maxalloc_cycles": st["fast_cycles"][5]}
if os.environ.get("KP_TIMING"):
    names = ["pop+stage", "existing", "sort", "inflight-commit", "templates", "record+bookkeeping", "inflight-prepass",
             "inflight-attempts"]
    tot = sum(st["phase_cycles"]) or 1
    out["phase_share"] = {k: round(v / tot, 4) for k, v in zip(names, st["phase_cycles"])}
    out["cycles_per_pop"] = round(tot / pops, 1)
    fp = max(1, st["fast_pods"])
    out["fast_cycles_per_fast_pod"] = dict(zip(["pop", "stage", "sort", "prepass", "attempts", "commit"],
                                               [round(c / fp, 1) for c in st["fast_cycles"]]))
    if "fine" in os.environ.get("KP_LIB", ""):  # FT_FINE build: attempt_cycles = the fast lane's finer split
        out["fast_fine_per_fast_pod"] = dict(zip(["window", "stage", "cursor", "sort", "nc-loads", "fits", "commit",
                                                   "existing-placed"], [round(c / fp, 1) for c in st["attempt_cycles"]]))
res = plan.run(read=True)
out["nodeclaims"] = len(res["nodeclaims"])
out["unschedulable"] = int((res["placement"] == -1).sum())
plan.close()
print(json.dumps(out), flush=True)
