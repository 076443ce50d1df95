"""Diagnostic: config 3's placements onto existing nodes — pods, distinct (node, shape) pairs, pods per node — from one
device Solve. usage: probe_ex_pairs.py [pods]"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "karpenter-provider-aws_amd"))
import numpy as np  # noqa: E402
import kpamd  # noqa: E402
from kpamd import catalog, synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
lib = kpamd.load_lib()
cat = catalog.build_catalog(lib)
prob = synth.config3(cat, n_pods=n)
ctx = kpamd.Context(0)
r = kpamd.Scheduler(ctx, prob).solve()
pl = np.asarray(r["placement"])
sh = np.asarray(prob.pod_shape)
ex = pl <= -2
pairs = {(int(a), int(b)) for a, b in zip(pl[ex], sh[ex])}
ncp = {(int(a), int(b)) for a, b in zip(pl[pl >= 0], sh[pl >= 0])}
print(json.dumps({"pods": n, "on_existing": int(ex.sum()), "existing_pairs": len(pairs),
                  "existing_nodes_used": len(set(pl[ex].tolist())), "on_nodeclaims": int((pl >= 0).sum()),
                  "nodeclaim_pairs": len(ncp), "shapes": int(sh.max()) + 1}))
