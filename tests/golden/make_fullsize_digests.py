"""Full-size parity fixtures (oracle results at BASELINE.json's sizes), generated in this container by the CPU oracle
(oracle/liboracle.so) on the committed generators, for the -m gpu tests in tests/test_fullsize_parity.py:

  config2-50000   Solve of config 2 at 50k pods: digest of the placement array and of the NodeClaims
                  (nodepool, pods in add order, options after OrderByPrice + Truncate, requirements)
  config2-burst-50000  config 2 with ReplicaSet bursts (synth.config2(burst=True): each deployment's pods created
                  within 2 s of its start): same digests
  config3-100000  Solve of config 3 at 100k pods (zone + hostname spread onto 5k existing nodes): same digests
  config5-100000  Solve of config 5 (20 weighted pools, GPU/Neuron pools) at 100k pods: 17.5k NodeClaims, so the
                  device's newNodeClaims order spills past its 8,192-entry LDS capacity on its own
  config5-limits-100000  config 5 at 100k pods with every pool's cpu limit divided by 10: the regime the 1M-pod burst
                  ends in (NodePool limits bind: subtractMax across 20 weighted pools, filterByRemainingResources on a
                  shrinking budget, failed pods cycling until a full pass makes no progress), 38.9 % unschedulable
  config5-1000000 config 5 at BASELINE's 1M pods (38.7 % unschedulable, 48k NodeClaims), when generated (hours of
                  oracle time: python tests/golden/make_fullsize_digests.py config5-1000000)
  config4-10000   computeConsolidation on the 10k-node config-4 cluster for every firstNConsolidationOption prefix
                  (candidates[0:mid+1], mid = 1..100) and 200 random subsets: every decision field
  general-2000    the bench's general-path leg: computeConsolidation on the 2,000-node spread cluster
                  (synth.spread_cluster: every other shape zone-spread) for the 100 firstNConsolidationOption prefixes
                  and 200 random subsets of 2..20 candidates (synth.consolidation_subsets seed 5), every decision field
  general-10000   the general path at config 4's size: the 10,000-node spread cluster, the 100 prefixes and 200
                  random subsets of 2..100 candidates (seed 6), every decision field (4 oracle processes, ~4 minutes)

Run from the repo root: python tests/golden/make_fullsize_digests.py [name ...]  (all: about 8 minutes); names given
regenerate only those entries.
"""
import hashlib
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "karpenter-provider-aws_amd"))

OUT = os.path.join(HERE, "fullsize_digests.json")


def solve_digest(res):
    """Stable digest of a Solve result (the device path returns the same structure)."""
    import numpy as np
    pl = hashlib.sha256(np.asarray(res["placement"], dtype=np.int32).tobytes()).hexdigest()
    h = hashlib.sha256()
    for n in res["nodeclaims"]:
        h.update(json.dumps([n["nodepool"], n["pods"], n["options"], n["n_remaining"], n["requirements"]],
                            sort_keys=True).encode())
    return {"placement_sha256": pl, "nodeclaims_sha256": h.hexdigest(), "nodeclaims": len(res["nodeclaims"]),
            "placed": int((np.asarray(res["placement"]) != -1).sum()),
            "on_existing": int((np.asarray(res["placement"]) <= -2).sum())}


def config4_subsets(cl):
    import numpy as np
    from kpamd import disruption
    cands = np.asarray(cl.candidates, dtype=np.uint32)
    pre = [[int(x) for x in cands[:m + 1]] for m in disruption.MultiNodeConsolidation.search_prefixes(len(cands))]
    offs, pos = disruption.random_subsets_csr(len(cands), 200, seed=4242)
    rnd = [[int(x) for x in cands[pos[offs[i]:offs[i + 1]]]] for i in range(200)]
    return pre, rnd


def sim_record(r):
    return [int(r["decision"]), int(r["nodepool"]), float(r["candidate_price"]).hex(), float(r["replacement_price"]).hex(),
            float(r["savings"]).hex(), int(r["n_options"]), int(r["n_pods"])]


def general_subsets(cl):
    import numpy as np
    from kpamd import disruption, synth
    cands = np.asarray(cl.candidates, dtype=np.uint32)
    pre = [[int(x) for x in cands[:m + 1]] for m in disruption.MultiNodeConsolidation.search_prefixes(len(cands))]
    rnd = [[int(x) for x in s] for s in synth.consolidation_subsets(cl, 200, seed=5, max_size=20, prefixes=False)]
    return pre, rnd


def general10k_subsets(cl):
    import numpy as np
    from kpamd import disruption, synth
    cands = np.asarray(cl.candidates, dtype=np.uint32)
    pre = [[int(x) for x in cands[:m + 1]] for m in disruption.MultiNodeConsolidation.search_prefixes(len(cands))]
    rnd = [[int(x) for x in s] for s in synth.consolidation_subsets(cl, 200, seed=6, max_size=100, prefixes=False)]
    return pre, rnd


def _general10k_worker(subs):
    import kpamd
    from kpamd import catalog, synth
    from oracle import pyoracle
    cl = synth.spread_cluster(catalog.build_catalog(kpamd.load_lib()), 10_000)
    res, _ = pyoracle.simulate_batch(cl, subs)
    return [sim_record(r) for r in res]


def _solves():
    from kpamd import synth
    return {"config2-50000": lambda cat: synth.config2(cat, n_pods=50_000, seed=2),
            "config2-burst-50000": lambda cat: synth.config2(cat, n_pods=50_000, seed=2, burst=True),
            "config3-100000": lambda cat: synth.config3(cat, n_pods=100_000),
            "config5-100000": lambda cat: synth.config5(cat, n_pods=100_000),
            "config5-limits-100000": lambda cat: synth.config5(cat, n_pods=100_000, limit_div=10),
            "config5-1000000": lambda cat: synth.config5(cat, n_pods=1_000_000)}


def main():
    import kpamd
    from kpamd import catalog, synth
    from oracle import pyoracle
    cat = catalog.build_catalog(kpamd.load_lib())
    SOLVES = {k: (lambda f: lambda: f(cat))(f) for k, f in _solves().items()}
    only = set(sys.argv[1:])
    out = json.load(open(OUT)) if os.path.exists(OUT) and only else {}
    for name, mk in SOLVES.items():
        if (only and name not in only) or (not only and name == "config5-1000000"):  # (hours: on request only)
            continue
        t = time.time()
        out[name] = solve_digest(pyoracle.solve(mk()))
        print(name, out[name], f"{time.time() - t:.1f}s", flush=True)
    if not only or "general-2000" in only:
        t = time.time()
        cl = synth.spread_cluster(cat, 2_000)
        pre, rnd = general_subsets(cl)
        res, _ = pyoracle.simulate_batch(cl, pre + rnd)
        out["general-2000"] = {"prefixes": [sim_record(r) for r in res[:len(pre)]],
                               "random": [sim_record(r) for r in res[len(pre):]]}
        print("general-2000", len(res), f"{time.time() - t:.1f}s", flush=True)
    if "general-10000" in only:  # (on request: minutes of oracle time)
        import multiprocessing as mp
        t = time.time()
        cl = synth.spread_cluster(cat, 10_000)
        pre, rnd = general10k_subsets(cl)
        allsubs = pre + rnd
        parts = [allsubs[i::4] for i in range(4)]
        with mp.get_context("spawn").Pool(4) as pool:
            outs = pool.map(_general10k_worker, parts)
        recs = [None] * len(allsubs)
        for i, o in enumerate(outs):
            recs[i::4] = o
        out["general-10000"] = {"prefixes": recs[:len(pre)], "random": recs[len(pre):]}
        print("general-10000", len(recs), f"{time.time() - t:.1f}s", flush=True)
    if only and "config4-10000" not in only:
        json.dump(out, open(OUT, "w"), indent=0)
        return
    t = time.time()
    cl = synth.config4(cat, n_nodes=10_000, seed=4)
    pre, rnd = config4_subsets(cl)
    res, _ = pyoracle.simulate_batch(cl, pre + rnd)
    out["config4-10000"] = {"prefixes": [sim_record(r) for r in res[:len(pre)]],
                            "random": [sim_record(r) for r in res[len(pre):]], "random_seed": 4242}
    print("config4", len(res), f"{time.time() - t:.1f}s", flush=True)
    json.dump(out, open(OUT, "w"), indent=0)


if __name__ == "__main__":
    main()
