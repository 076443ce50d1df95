"""Diagnostic: run kp_solve on a config (default config 2, 50k pods) `reps` times — a short program for
rocprofv3 --pmc passes over solve_kernel. usage: solve_once.py [config] [pods] [reps]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "karpenter-provider-aws_amd"))
import kpamd  # noqa: E402
from kpamd import catalog, synth  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "2"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 50000
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 1
lib = kpamd.load_lib()
cat = catalog.build_catalog(lib)
prob = {"1": lambda: synth.config1(cat, n_pods=n), "2": lambda: synth.config2(cat, n_pods=n, seed=2),
        "3": lambda: synth.config3(cat, n_pods=n), "5": lambda: synth.config5(cat, n_pods=n)}[cfg]()
ctx = kpamd.Context(0)
import _ov  # noqa: E402  (tools only: diagnostic variables -> kp_overrides)
_ov.apply(ctx)
sched = kpamd.Scheduler(ctx, prob)
for _ in range(reps):
    r = sched.solve(read=False)
print(r["stats"]["solve_kernel_ms"], r["stats"]["fast_pods"])
