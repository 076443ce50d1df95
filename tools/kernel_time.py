"""solve_kernel time of one config (default 2): 1 warmup + 5 timed kp_solve calls; prints the kernel ms (min, mean),
the per-Solve prepare and the whole call (means).
Works with any libkp build selected by KP_LIB (older ABIs included). usage: kernel_time.py [2|3|5] [pods]"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "karpenter-provider-aws_amd"))
import kpamd  # noqa: E402
from kpamd import catalog, synth  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "2"
if cfg.endswith("-off"):  # the fast lane without its continuation variant (kp_solve's choice overridden)
    os.environ["KP_CONT"] = "0"
    cfg = cfg[:-4]
elif cfg.endswith("-on"):  # the fast lane with its continuation variant
    os.environ["KP_CONT"] = "1"
    cfg = cfg[:-3]
n = int(sys.argv[2]) if len(sys.argv) > 2 else {"2": 50000, "2b": 50000, "3": 100000, "5": 100000}[cfg]
lib = kpamd.load_lib()
cat = catalog.build_catalog(lib)
prob = {"2": lambda: synth.config2(cat, n_pods=n, seed=2), "2b": lambda: synth.config2(cat, n_pods=n, seed=2, burst=True),
        "3": lambda: synth.config3(cat, n_pods=n), "5": lambda: synth.config5(cat, n_pods=n)}[cfg]()
ctx = kpamd.Context(0)
import _ov  # noqa: E402  (tools only: diagnostic variables -> kp_overrides)
_ov.apply(ctx)
sched = kpamd.Scheduler(ctx, prob)
import time  # noqa: E402
sched.solve(read=False)
ks, ps, ws = [], [], []
for _ in range(5):
    t0 = time.perf_counter()
    st = sched.solve(read=False)["stats"]
    ws.append((time.perf_counter() - t0) * 1e3)
    ks.append(st["solve_kernel_ms"])
    ps.append(st["prepare_ms"])
print(json.dumps({"min_ms": round(min(ks), 2), "mean_ms": round(sum(ks) / len(ks), 2),
                  "prep_ms": round(sum(ps) / len(ps), 2), "step_ms": round(sum(ws) / len(ws), 2)}))
