"""Device launch == oracle launch on many random reservation catalogues (a wider sweep than the test's 4 seeds)."""
import sys
sys.path.insert(0, ".")
sys.path.insert(0, "tests")
sys.path.insert(0, "karpenter-provider-aws_amd")
import kpamd
from kpamd import catalog as cmod
from oracle import pyoracle
from test_reserved_offerings import reserved_catalogue, reserved_requests

ctx = kpamd.Context(0)
n_bad = n_res = n_req = 0
for seed in range(int(sys.argv[1]) if len(sys.argv) > 1 else 16):
    cat = reserved_catalogue(None, 200 + 40 * seed, 1000 + seed)
    reqs = reserved_requests(cat, 200, 2000 + seed)
    zones = [cmod.ZONES, cmod.ZONES[:1], cmod.ZONES[1:], []][seed % 4]
    ch = kpamd.Catalog(ctx, cat)
    plan = kpamd.LaunchPlan(ctx, ch, reqs, zones, max_types=[60, 5, 1, 200][seed % 4])
    got, _ = plan.run(read=True)
    plan.close()
    ch.close()
    want = pyoracle.launch_select(cat, reqs, zones, max_types=[60, 5, 1, 200][seed % 4])
    bad = [i for i, (g, w) in enumerate(zip(got, want)) if g != w]
    n_bad += len(bad)
    n_res += sum(g["capacity_type"] == "reserved" for g in got)
    n_req += len(reqs)
    print(f"seed {seed}: {len(reqs)} requests, {len(bad)} mismatches, reserved {sum(g['capacity_type'] == 'reserved' for g in got)}",
          flush=True)
    for i in bad[:2]:
        print("  device", got[i], "\n  oracle", want[i])
print(f"total {n_req} requests, {n_res} reserved launches, {n_bad} mismatches")
ctx.close()
sys.exit(1 if n_bad else 0)
