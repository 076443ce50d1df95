"""Feasibility leg probe: median device time of kp_filter_run over pairwise-distinct rows (the bench's roofline leg),
per variant given on the command line as NAME=ENV1=V1,ENV2=V2 (plans are prepared after setting the env)."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "karpenter-provider-aws_amd"))
import kpamd  # noqa: E402
from kpamd import catalog, synth  # noqa: E402

rows = int(os.environ.get("FEAS_ROWS", "50000"))
lib = kpamd.load_lib()
cat = catalog.build_catalog(lib)
ctx = kpamd.Context(0)
import _ov  # noqa: E402  (tools only: diagnostic variables -> kp_overrides)
_ov.apply(ctx)
ch = kpamd.Catalog(ctx, cat)
qs = synth.distinct_queries(cat, rows)
out = {}
KNOBS = ("KP_FEAS_GLOBAL", "KP_FEAS_ONE_ROW", "KP_FEAS_BLOCKS", "KP_FEAS_TEMPORAL")
for spec in sys.argv[1:] or ["lds"]:
    name, _, envs = spec.partition("=")
    for k in KNOBS:
        os.environ.pop(k, None)
    for kv in filter(None, envs.split(",")):
        k, _, v = kv.partition("=")
        os.environ[k] = v
    _ov.apply(ctx)
    for cheapest in ((True,) if os.environ.get("FEAS_CHEAPEST_ONLY") else (True, False)):
        fp = kpamd.FilterPlan(ctx, ch, qs, cheapest=cheapest)
        fp.run()
        sts = [fp.run() for _ in range(int(os.environ.get("FEAS_REPS", "10")))]
        ms = sorted(x["device_ms"] for x in sts)
        if os.environ.get("KP_TIMING"):
            out[f"{name}{'' if cheapest else '_nocheapest'}_phases"] = sts[-1]["phase_cycles"][:4]
        fp.close()
        out[f"{name}{'' if cheapest else '_nocheapest'}"] = round(ms[len(ms) // 2], 4)
print(json.dumps(out), flush=True)
