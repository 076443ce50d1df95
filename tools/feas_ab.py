"""Feasibility leg device times (median of 15) for the library KP_LIB selects: the price-row form and the compact form
over 50k pairwise-distinct rows (the bench's legs). usage: KP_LIB=... feas_ab.py"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "karpenter-provider-aws_amd"))
import kpamd  # noqa: E402
from kpamd import catalog, synth  # noqa: E402

lib = kpamd.load_lib()
cat = catalog.build_catalog(lib)
ctx = kpamd.Context(0)
ch = kpamd.Catalog(ctx, cat)
qs = synth.distinct_queries(cat, 50000)
out = {}
fp = kpamd.FilterPlan(ctx, ch, qs, cheapest=True)
fp.run()
ms = sorted(fp.run()["device_ms"] for _ in range(15))
out["rows_ms"] = round(ms[7], 4)
fp.close()
fp = kpamd.FilterPlan(ctx, ch, qs, cheapest="compact")
fp.run_compact(read=False)
ms = sorted(fp.run_compact(read=False)["device_ms"] for _ in range(15))
out["compact_ms"] = round(ms[7], 4)
fp.close()
print(json.dumps(out))
