"""Times kp_cluster_simulate on a config-4 cluster (first numbers; bench.py carries the contract line)."""
import json
import sys
import time

sys.path.insert(0, "karpenter-provider-aws_amd")
import kpamd  # noqa: E402
from kpamd import catalog as kc, synth  # noqa: E402

n_nodes = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
n_rand = int(sys.argv[2]) if len(sys.argv) > 2 else 20000
lib = kpamd.load_lib()
cat = kc.build_catalog(lib)
t = time.time()
cl = synth.config4(cat, n_nodes=n_nodes, seed=4)
subs = synth.consolidation_subsets(cl, n_rand, seed=44)
gen_s = time.time() - t
ctx = kpamd.Context(0)
t = time.time()
plan = kpamd.ClusterPlan(ctx, cl)
prep_s = time.time() - t
out = {"nodes": n_nodes, "pods": int(len(cl.pod_shape)), "subsets": len(subs), "gen_s": gen_s, "prepare_s": prep_s}
for rep in range(3):
    t = time.time()
    res, st = plan.simulate(subs, raw=True)
    wall = time.time() - t
    out[f"run{rep}"] = {"wall_s": wall, "kernel_ms": st["solve_kernel_ms"], "sims_per_s": len(subs) / (st["solve_kernel_ms"] / 1e3),
                        "pops": st["pops"], "attempts": st["attempts"], "words": st["phase_cycles"][0]}
from collections import Counter  # noqa: E402
out["decisions"] = dict(Counter(int(res[i].decision) for i in range(len(subs))))
print(json.dumps(out))
