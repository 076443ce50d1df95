"""Run-length commit probe: for config 2 with uniform creation times and with per-deployment bursts,
the runs of one shape-level in Queue order and how often a run's consecutive pods land on the same NodeClaim (a
run-length commit places a run's pods with one Add only when they do). Device Solve (GPU) or the oracle (CPU: --oracle).
JSON to stdout."""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "karpenter-provider-aws_amd"))
sys.path.insert(0, REPO)
import kpamd  # noqa: E402
from kpamd import catalog, synth  # noqa: E402


def queue_order(prob):
    req = lambda s, k: prob.shapes[s].requests.get(k, 0)
    keys = [(-req(int(prob.pod_shape[p]), "cpu"), -req(int(prob.pod_shape[p]), "memory"), int(prob.pod_creation[p]),
             int(prob.pod_uid[p]), p) for p in range(prob.n_pods)]
    return [k[-1] for k in sorted(keys)]


def main():
    use_oracle = "--oracle" in sys.argv
    n = int(os.environ.get("RL_PODS", "50000"))
    lib = kpamd.load_lib()
    cat = catalog.build_catalog(lib)
    ctx = None if use_oracle else kpamd.Context(0)
    for burst in (False, True):
        prob = synth.config2(cat, n_pods=n, seed=2, burst=burst)
        if use_oracle:
            from oracle import pyoracle
            res = pyoracle.solve(prob)
            ms = res["stats"]["host_ms"]
        else:
            sched = kpamd.Scheduler(ctx, prob)
            sched.solve(read=False)
            res = sched.solve(read=True)
            ms = res["stats"]["solve_kernel_ms"]
        q = queue_order(prob)
        shp = prob.pod_shape[q]
        pl = res["placement"][q]
        runs = np.split(np.arange(len(q)), np.nonzero(np.diff(shp))[0] + 1)
        same = sum(int(pl[i] == pl[i - 1] and pl[i] >= 0) for r in runs for i in r[1:])
        pairs = sum(len(r) - 1 for r in runs)
        print(json.dumps({"burst": burst, "pods": n, "runs": len(runs), "mean_run": round(len(q) / len(runs), 2),
                          "consecutive_same_nodeclaim": same, "consecutive_pairs": pairs,
                          "share_same": round(same / max(1, pairs), 3), "solve_ms": round(ms, 2),
                          "us_per_pod": round(1000 * ms / n, 3), "nodeclaims": len(res["nodeclaims"]),
                          "fast_pods": res["stats"].get("fast_pods")}), flush=True)


if __name__ == "__main__":
    main()
