"""Diagnostic: per-phase cycle split of solve_kernel (KP_TIMING=1). usage: profile_solve.py [config] [pods]
The fast lane's phases need the diagnostic build: KP_LIB=tools/fine/libkp.so (tools/build_fine.sh)."""
import json
import os
import sys

os.environ["KP_TIMING"] = "1"
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "karpenter-provider-aws_amd"))
import kpamd  # noqa: E402
from kpamd import catalog, synth  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "2"
n = int(sys.argv[2]) if len(sys.argv) > 2 else {"2": 50000, "2b": 50000, "3": 100000, "5": 300000}[cfg]
lib = kpamd.load_lib()
cat = catalog.build_catalog(lib)
prob = {"2": lambda: synth.config2(cat, n_pods=n, seed=2), "2b": lambda: synth.config2(cat, n_pods=n, seed=2, burst=True), "3": lambda: synth.config3(cat, n_pods=n, n_deployments=int(os.environ.get("KP_C3_DEPLOYMENTS", "1000"))),
        "5": lambda: synth.config5(cat, n_pods=n)}[cfg]()
ctx = kpamd.Context(0)
import _ov  # noqa: E402  (tools only: diagnostic variables -> kp_overrides)
_ov.apply(ctx)
sched = kpamd.Scheduler(ctx, prob)
sched.solve(read=False)
r = sched.solve(read=True)
st = r["stats"]
names = ["pop+stage", "existing", "sort", "inflight-commit", "templates", "record+bookkeeping", "inflight-prepass",
         "inflight-attempts"]
tot = sum(st["phase_cycles"]) or 1
out = {"config": cfg, "pods": n, "solve_kernel_ms": st["solve_kernel_ms"], "attempts": st["attempts"],
       "pops": st["pops"], "nodeclaims": len(r["nodeclaims"]), "attempts_per_pop": st["attempts"] / max(1, st["pops"]),
       "phase_share": {k: round(v / tot, 4) for k, v in zip(names, st["phase_cycles"])},
       "cycles_per_pop": tot / max(1, st["pops"]), "scanned_per_pop": st["scanned"] / max(1, st["pops"]),
       "cursor_start_per_pop": st["cursor_starts"] / max(1, st["pops"])}
ac = st["attempt_cycles"]
if ac[5]:
    out["attempt_cycles_per_attempt"] = {k: round(v / ac[5], 1) for k, v in
                                         zip(["merge", "pod-key-rows", "fits-rows", "offer-rows+row-loads", "minvalues"], ac[:5])}
    out["attempts_timed"] = ac[5]
out["fast_pods"] = st["fast_pods"]
out["slow_sorts"] = st["slow_sorts"]
fc = st["fast_cycles"]
if os.environ.get("EX_DIAG"):  # variant build: the existing-node scan in place of the fast-lane phases
    out["existing_diag_per_pop"] = {k: round(v / max(1, st["pops"]), 2) for k, v in
                                    zip(["staging_cycles", "prepass_cycles", "attempt_cycles", "scans", "cycles", "eval_cycles"], fc)}
if os.environ.get("FX_DIAG"):  # variant build: the fast lane's existing-node scans (counts over the Solve)
    out["fast_existing_scans"] = dict(zip(["scans", "rounds", "placed", "skipped", "failed", "bailed"], fc))
if os.environ.get("SORT_DIAG"):  # variant build: the full path's sort split in place of the fast-lane phases
    out["sort_diag_per_pop"] = {k: round(v / max(1, st["pops"]), 2) for k, v in
                                zip(["decision_cycles", "shift_cycles", "shifted", "mode1", "mode2", "mode3"], fc)}
if sum(fc):
    out["fast_cycles_per_fast_pod"] = {k: round(v / max(1, st["fast_pods"]), 1) for k, v in
                                       zip(["pop", "stage", "sort", "prepass", "attempts", "commit"], fc)}
out["fast_fine_per_fast_pod"] = dict(zip(["window", "stage", "cursor", "sort", "nc-loads", "fits", "commit",
                                          "existing-placed"], [round(v / max(1, st["fast_pods"]), 1) for v in ac]))
# (FT_FINE builds: probes 6..13; "existing-placed" is FT(0) to a placement on an existing node, those pods only)
out["fast_bails"] = dict(zip(["ineligible", "spilled", "shift", "scan", "merge", "minvalues", "none", "-"],
                             st["fast_bails"]))
print(json.dumps(out))
