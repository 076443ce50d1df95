"""General-path consolidation at config 4's size: the 10,000-node spread cluster
(synth.spread_cluster), the 100 firstNConsolidationOption prefixes + N random subsets of 2..100 candidates through
kp_consolidate_argmin, timed with and without kp_cluster_prepare; KP_HOST_TIMING=1 prints the host/device split.
usage: python tools/general_scale.py [n_nodes] [n_random] [--digest]  (writes gpurun_out/general_scale.json)"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "karpenter-provider-aws_amd"))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))


def main():
    import numpy as np
    import kpamd
    from kpamd import catalog as kc, disruption, synth
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    n_nodes = int(args[0]) if args else 10_000
    n_random = int(args[1]) if len(args) > 1 else 2000
    lib = kpamd.load_lib()
    cat = kc.build_catalog(lib)
    ctx = kpamd.Context(0)
    import _ov  # noqa: E402  (tools only: diagnostic variables -> kp_overrides)
    _ov.apply(ctx)
    t0 = time.perf_counter()
    cl = synth.spread_cluster(cat, n_nodes)
    gen_s = time.perf_counter() - t0
    cands = np.asarray(cl.candidates, dtype=np.uint32)
    mids = disruption.MultiNodeConsolidation.search_prefixes(len(cands))
    subs = [list(cands[:m + 1]) for m in mids]
    subs += synth.consolidation_subsets(cl, n_random, seed=6, max_size=100, prefixes=False)
    offs = np.zeros(len(subs) + 1, dtype=np.uint32)
    offs[1:] = np.cumsum([len(x) for x in subs])
    flat = np.concatenate([np.asarray(x, dtype=np.uint32) for x in subs])
    out = {"nodes": n_nodes, "pods": int(len(cl.pod_shape)), "subsets": len(subs), "gen_s": round(gen_s, 2)}
    t0 = time.perf_counter()
    plan = kpamd.ClusterPlan(ctx, cl)
    out["prepare_s"] = round(time.perf_counter() - t0, 3)
    print("prepare", out["prepare_s"], flush=True)
    plan.argmin(offs[:min(len(subs), 8192) + 1], flat)  # warmup: the batch layout and both slots' arenas (steady state)
    t0 = time.perf_counter()
    choice, _, st = plan.argmin(offs, flat)
    el = time.perf_counter() - t0
    out.update({"elapsed_s": round(el, 3), "sims_per_s": round(len(subs) / el, 1),
                "sims_per_s_incl_prepare": round(len(subs) / (el + out["prepare_s"]), 1),
                "decisions": choice["counts"], "stats": {k: st[k] for k in ("device_ms", "host_ms") if k in st}})
    print(json.dumps(out), flush=True)
    if "--digest" in sys.argv:  # the committed oracle digest of the 100 prefixes + 200 random subsets (seed 6)
        import make_fullsize_digests as mk
        pre, rnd = mk.general10k_subsets(cl)
        res, _ = plan.simulate(pre + rnd)
        got = [mk.sim_record(r) for r in res]
        want = json.load(open(os.path.join(ROOT, "tests", "golden", "fullsize_digests.json"))).get("general-10000")
        if want:
            out["digest_equal"] = got == want["prefixes"] + want["random"]
            print("digest equal:", out["digest_equal"], flush=True)
    plan.close()
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    json.dump(out, open(os.path.join(ROOT, "gpurun_out", "general_scale.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
