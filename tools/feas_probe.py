"""Feasibility-kernel probe: device time of kp_filter_run with / without the cheapest-price output, at two row
counts (separates the output stream from the per-row work)."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "karpenter-provider-aws_amd"))
import kpamd  # noqa: E402
from kpamd import catalog, synth  # noqa: E402

lib = kpamd.load_lib(*(sys.argv[1:2]))
cat = catalog.build_catalog(lib)
ctx = kpamd.Context(0)
ch = kpamd.Catalog(ctx, cat)
out = {}
for n in (5000, 50000):
    prob = synth.config2(cat, n_pods=n, seed=2)
    qs = kpamd.pod_queries(prob)
    for cheapest in (False, True):
        fp = kpamd.FilterPlan(ctx, ch, qs, cheapest=cheapest)
        fp.run()
        ms = sorted(fp.run()["device_ms"] for _ in range(10))
        fp.close()
        out[f"rows{n}_cheapest{int(cheapest)}"] = round(ms[len(ms) // 2], 4)
print(json.dumps(out))
