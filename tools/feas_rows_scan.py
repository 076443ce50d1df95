"""Compact feasibility device time against the row count (multiples of one full round of wave slots: 256 CUs x 24
waves x 4 rows = 24,576 rows), to see whether the last partial round of quads sets the time. usage: feas_rows_scan.py"""
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
qs_all = synth.distinct_queries(cat, 61440)
out = {}
for rows in (12288, 24576, 36864, 45056, 49152, 50000, 53248, 61440):
    qs = qs_all[:rows]
    fp = kpamd.FilterPlan(ctx, ch, qs, cheapest="compact")
    fp.run_compact(read=False)
    ms = sorted(fp.run_compact(read=False)["device_ms"] for _ in range(15))
    fp.close()
    out[rows] = round(ms[len(ms) // 2], 4)
    print(rows, out[rows], file=sys.stderr, flush=True)
print(json.dumps(out))
