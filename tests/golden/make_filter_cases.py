"""Transcribes the kept/rejected expectations of R:pkg/providers/instance/filter/filter_test.go:47-629
into data (tests/golden/filter_cases.json). Instance types are built the way the test helpers build them
(makeInstanceType/makeOffering/withZone/withPrice, R:filter_test.go:633-743): empty overhead, capacity only
what withResource sets, offerings with only capacity-type (+zone/price when given). The reserved-capacity
filters' cases (CapacityReservationType / CapacityBlock / ReservedOffering, R:filter_test.go:130-396) are transcribed
in tests/test_reserved_offerings.py instead (they need reservation ids / types on the offerings).
"""
import json
import os

CT = "karpenter.sh/capacity-type"
Z = "topology.kubernetes.io/zone"


def it(name, reqs=(), cap=None, offs=()):
    return {"name": name, "requirements": [list(r) for r in reqs], "capacity": cap or {}, "offerings": list(offs)}


def off(ct, avail, zone=None, price=0.0):
    return {"capacity_type": ct, "available": avail, "zone": zone, "price": price}


cases = []
# CompatibleAvailableFilter (R:filter_test.go:48-128)
q = [[Z, "In", ["zone-1a"]]]
cases.append({"name": "compatible-by-requirements", "filter": "compatible_available", "requirements": q,
              "requests": {"cpu": 1000}, "types": [
                  it("compatible-instance", [(Z, "In", ["zone-1a"])], {"cpu": 2000}, [off("on-demand", True, "zone-1a")]),
                  it("incompatible-instance", [(Z, "In", ["zone-1b"])], {"cpu": 2000}, [off("on-demand", True, "zone-1b")])],
              "kept": ["compatible-instance"]})
cases.append({"name": "compatible-by-requests", "filter": "compatible_available", "requirements": q,
              "requests": {"cpu": 1000}, "types": [
                  it("compatible-instance", [(Z, "In", ["zone-1a"])], {"cpu": 2000}, [off("on-demand", True, "zone-1a")]),
                  it("incompatible-instance", [(Z, "In", ["zone-1a"])], {"cpu": 500}, [off("on-demand", True, "zone-1a")])],
              "kept": ["compatible-instance"]})
cases.append({"name": "compatible-available", "filter": "compatible_available", "requirements": q,
              "requests": {"cpu": 1000}, "types": [
                  it("available-instance", [(Z, "In", ["zone-1a"])], {"cpu": 2000}, [off("on-demand", True, "zone-1a")]),
                  it("unavailable-instance", [(Z, "In", ["zone-1a"])], {"cpu": 2000}, [off("on-demand", False, "zone-1a")])],
              "kept": ["available-instance"]})
# ExoticInstanceTypeFilter (R:filter_test.go:398-469)
EXOTIC = ["nvidia.com/gpu", "amd.com/gpu", "aws.amazon.com/neuron", "aws.amazon.com/neuroncore", "habana.ai/gaudi"]
NORMAL = ["cpu", "memory", "ephemeral-storage", "pods", "vpc.amazonaws.com/pod-eni", "vpc.amazonaws.com/efa"]
for r in EXOTIC:
    cases.append({"name": f"exotic-rejects-{r}", "filter": "exotic", "requirements": [],
                  "types": [it("generic-instance-type"), it("exotic-instance-type", cap={r: 1000})],
                  "kept": ["generic-instance-type"]})
for r in NORMAL:
    cases.append({"name": f"exotic-keeps-{r}", "filter": "exotic", "requirements": [],
                  "types": [it("generic-instance-type", cap={r: 1000}), it("exotic-instance-type", cap={EXOTIC[0]: 1000})],
                  "kept": ["generic-instance-type"]})
SIZE = "karpenter.k8s.aws/instance-size"
cases.append({"name": "exotic-rejects-metal", "filter": "exotic", "requirements": [],
              "types": [it("generic-instance-type"), it("generic-instance-type-metal", [(SIZE, "In", ["metal"])])],
              "kept": ["generic-instance-type"]})
cases.append({"name": "exotic-falls-back", "filter": "exotic", "requirements": [],
              "types": [it("exotic-instance-type", cap={EXOTIC[0]: 1000}),
                        it("generic-instance-type-metal", [(SIZE, "In", ["metal"])])],
              "kept": ["exotic-instance-type", "generic-instance-type-metal"]})
cases.append({"name": "exotic-minvalues", "filter": "exotic",
              "requirements": [["node.kubernetes.io/instance-type", "Exists", [], 2]],
              "types": [it("generic-instance-type"), it("exotic-instance-type", cap={EXOTIC[0]: 1000})],
              "kept": ["generic-instance-type", "exotic-instance-type"]})
# SpotInstanceFilter (R:filter_test.go:471-630)
cases.append({"name": "spot-rejects-expensive", "filter": "spot", "requirements": [[CT, "Exists", []]], "types": [
    it("expensive-od-instance", offs=[off("on-demand", True, price=15.0), off("on-demand", True, price=15.0)]),
    it("od-instance", offs=[off("on-demand", True, price=5.0), off("on-demand", True, price=10.0)]),
    it("cheap-spot-instance", offs=[off("spot", True, price=1.0), off("spot", True, price=2.0)]),
    it("mixed-spot-instance", offs=[off("spot", True, price=1.0), off("spot", True, price=10.0)]),
    it("mixed-unavailable-spot-instance", offs=[off("spot", False, price=1.0), off("spot", True, price=10.0)]),
    it("expensive-spot-instance", offs=[off("spot", True, price=10.0), off("spot", True, price=10.0)])],
    "kept": ["expensive-od-instance", "od-instance", "cheap-spot-instance", "mixed-spot-instance"]})
cases.append({"name": "spot-zonal", "filter": "spot", "requirements": [[CT, "Exists", []], [Z, "In", ["zone-1a", "zone-1b"]]],
              "types": [
    it("expensive-od-instance", offs=[off("on-demand", True, "zone-1a", 15.0), off("on-demand", True, "zone-1b", 15.0)]),
    it("od-instance", offs=[off("on-demand", True, "zone-1a", 5.0), off("on-demand", True, "zone-1b", 10.0)]),
    it("cheap-spot-instance", offs=[off("spot", True, "zone-1a", 1.0), off("spot", True, "zone-1b", 2.0)]),
    it("mixed-spot-instance", offs=[off("spot", True, "zone-1a", 1.0), off("spot", True, "zone-1b", 10.0)]),
    it("mixed-compatible-available-spot-instance", offs=[off("spot", True, "zone-1a", 1.0), off("spot", True, "zone-1c", 10.0)]),
    it("reserved-instance", offs=[off("spot", True, "zone-1a", 10.0), off("spot", True, "zone-1b", 10.0),
                                  off("reserved", True, "zone-1b")]),
    it("mixed-unavailable-spot-instance", offs=[off("spot", False, "zone-1a", 1.0), off("spot", True, "zone-1b", 10.0)]),
    it("mixed-compatible-unavailable-spot-instance", offs=[off("spot", True, "zone-1a", 10.0), off("spot", True, "zone-1c", 1.0)]),
    it("expensive-spot-instance", offs=[off("spot", True, "zone-1a", 10.0), off("spot", True, "zone-1b", 10.0)])],
    "kept": ["expensive-od-instance", "od-instance", "cheap-spot-instance", "mixed-spot-instance",
             "mixed-compatible-available-spot-instance", "reserved-instance"]})
three = [it("od-instance", offs=[off("on-demand", True, price=5.0)]),
         it("cheap-spot-instance", offs=[off("spot", True, price=1.0)]),
         it("expensive-spot-instance", offs=[off("spot", True, price=10.0)])]
cases.append({"name": "spot-only-spot-compatible", "filter": "spot", "requirements": [[CT, "In", ["spot"]]],
              "types": three, "kept": ["od-instance", "cheap-spot-instance", "expensive-spot-instance"]})
cases.append({"name": "spot-minvalues", "filter": "spot",
              "requirements": [[CT, "Exists", []], ["node.kubernetes.io/instance-type", "Exists", [], 2]],
              "types": three, "kept": ["od-instance", "cheap-spot-instance", "expensive-spot-instance"]})

out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "filter_cases.json")
json.dump(cases, open(out, "w"), indent=1)
print(len(cases), "cases ->", out)
