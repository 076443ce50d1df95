"""Post-Solve instance filters pinned by R:pkg/providers/instance/filter/filter_test.go (kept sets).

Oracle: CompatibleAvailable / Spot / Exotic. Device: CompatibleAvailableFilter through
kp_filter_compatible_available (the batched feasibility kernel), gpu-marked.
"""
import json
import os

import pytest

from kpamd.model import InstanceType, Offering

CASES = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "filter_cases.json")))


def mk_types(case):
    out = []
    for t in case["types"]:
        offs = [Offering(o["capacity_type"], o["zone"], None, float(o["price"]), bool(o["available"]))
                for o in t["offerings"]]
        out.append(InstanceType(t["name"], [tuple(r) for r in t["requirements"]], dict(t["capacity"]), {}, offs))
    return out


def reqs(case):
    return [tuple(r) for r in case["requirements"]]


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_oracle_filter_cases(case):
    from oracle import pyoracle
    types = mk_types(case)
    if case["filter"] == "compatible_available":
        kept, _ = pyoracle.compatible_available_filter(types, reqs(case), case["requests"])
    elif case["filter"] == "spot":
        kept = pyoracle.spot_filter(types, reqs(case))
    else:
        kept = pyoracle.exotic_filter(types, reqs(case))
    assert sorted(t.name for t, k in zip(types, kept) if k) == sorted(case["kept"])


@pytest.mark.gpu
@pytest.mark.parametrize("case", [c for c in CASES if c["filter"] == "compatible_available"],
                         ids=[c["name"] for c in CASES if c["filter"] == "compatible_available"])
def test_device_compatible_available_cases(ctx, case):
    import kpamd
    types = mk_types(case)
    cat = kpamd.Catalog(ctx, types)
    kept, _, _ = kpamd.compatible_available_filter(ctx, cat, [(reqs(case), case["requests"])])
    assert sorted(t.name for t, k in zip(types, kept[0]) if k) == sorted(case["kept"])
