"""kp_cluster_prepare's cost split on the general-path cluster (synth.spread_cluster) and on config 4: the catalogue
upload, the Python marshalling into kp_cluster (abi.build_cluster) and the C call itself, timed apart.
usage: prep_probe.py [n_nodes]   (KP_HOST_TIMING=1: libkp prints its own phases)"""
import ctypes as C
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "karpenter-provider-aws_amd"))
import kpamd  # noqa: E402
from kpamd import abi, catalog, synth  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000
    lib = kpamd.load_lib()
    cat = catalog.build_catalog(lib)
    ctx = kpamd.Context(0)
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import _ov
    _ov.apply(ctx)
    out = {}
    for name, cl in (("general", synth.spread_cluster(cat, n)), ("config4", synth.config4(cat, n_nodes=n, seed=4))):
        for rep in range(2):
            t0 = time.perf_counter()
            cats = [kpamd.Catalog(ctx, c) for c in cl.catalogs]
            t1 = time.perf_counter()
            arena = abi.Arena()
            cs = abi.build_cluster(arena, cl, catalog_handles=[c.h.value for c in cats])
            t2 = time.perf_counter()
            h = C.c_void_p()
            rc = ctx.lib.kp_cluster_prepare(ctx.h, C.byref(cs), C.byref(h))
            t3 = time.perf_counter()
            assert rc == 0, rc
            ctx.lib.kp_cluster_plan_destroy(h)
            for c in cats:
                c.close()
            out[f"{name}_{rep}"] = {"catalog_s": round(t1 - t0, 3), "marshal_s": round(t2 - t1, 3),
                                    "kp_cluster_prepare_s": round(t3 - t2, 3)}
            print(name, out[f"{name}_{rep}"], file=sys.stderr, flush=True)
    ctx.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
