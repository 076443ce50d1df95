"""Diagnostic: per-phase cycle split of solve_kernel (KP_TIMING=1) on the config-2 workload."""
import json
import os
import sys

os.environ["KP_TIMING"] = "1"
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "karpenter-provider-aws_amd"))
import kpamd  # noqa: E402
from kpamd import catalog, synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 50000
lib = kpamd.load_lib()
cat = catalog.build_catalog(lib)
prob = synth.config2(cat, n_pods=n, seed=2)
ctx = kpamd.Context(0)
plan = kpamd.Scheduler(ctx, prob).prepare()
plan.run(read=False)
r = plan.run(read=True)
st = r["stats"]
names = ["pop+stageB", "existing", "sort", "inflight-commit", "templates", "bookkeeping", "inflight-prepass", "inflight-attempts"]
tot = sum(st["phase_cycles"]) or 1
out = {"pods": n, "solve_kernel_ms": st["solve_kernel_ms"], "attempts": st["attempts"], "pops": st["pops"],
       "nodeclaims": len(r["nodeclaims"]), "attempts_per_pod": st["attempts"] / n,
       "phase_share": {k: round(v / tot, 4) for k, v in zip(names, st["phase_cycles"]) },
       "cycles_per_pod": tot / n}
print(json.dumps(out))
