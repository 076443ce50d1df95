"""Full-size CPU baselines: the oracle (oracle/liboracle.so, single thread) timed on the whole
configs the bench line quotes — config 2 (50k pods), config 3 (100k pods onto 5k existing nodes), config 5 (1M pods,
20 pools, limits binding) — with the machine named. Writes profiles/r05/cpu_fullsize.json, which bench.py reports as
cpu_baseline.full_size beside the bounded sample it times live. Test/bench infrastructure only (the oracle is the
checker and the CPU baseline, never the product).
usage: python tools/cpu_fullsize.py [config2 config3 config5]"""
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "karpenter-provider-aws_amd"))
sys.path.insert(0, ROOT)


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor()


def main(which):
    import kpamd
    from kpamd import catalog as kc, synth
    from oracle import pyoracle
    lib = kpamd.load_lib()
    cat = kc.build_catalog(lib)
    out_path = os.path.join(ROOT, "profiles", "r05", "cpu_fullsize.json")
    out = json.load(open(out_path)) if os.path.exists(out_path) else {}
    gens = {"config2": lambda: synth.config2(cat), "config3": lambda: synth.config3(cat),
            "config5": lambda: synth.config5(cat)}
    for name in which:
        prob = gens[name]()
        t0 = time.perf_counter()
        res = pyoracle.solve(prob)
        dt = time.perf_counter() - t0
        placed = int(sum(1 for p in res["placement"] if p != -1))
        out[name] = {"pods": prob.n_pods, "placed": placed, "seconds": round(dt, 2),
                     "pods_per_s": round(prob.n_pods / dt, 1), "placed_per_s": round(placed / dt, 1),
                     "threads": 1, "cpu": cpu_model(), "host": platform.node()}
        print(name, out[name], flush=True)
        json.dump(out, open(out_path, "w"), indent=1)


if __name__ == "__main__":
    main(sys.argv[1:] or ["config2", "config3", "config5"])
