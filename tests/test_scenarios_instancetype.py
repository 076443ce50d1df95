"""Reference Solve scenarios of the instancetype suite, transcribed (a13/a2/a3 of SURVEY §8): each runs
ExpectProvisioned (Solve + launch selection through tests/scenarios.py) on the oracle and, under -m gpu, on the device,
with the suite's fake 16-type catalogue (R:pkg/fake/zz_generated.describe_instance_types.go; EC2 facts from the
committed docs table), its on-demand NodePool (R:pkg/providers/instancetype/suite_test.go:150-171) and, where the
suite applies it, its Windows 2022 NodePool / EC2NodeClass (:172-216).

  :223-283  every well-known label (and the normalized deprecated ones) as a single-label nodeSelector: scheduled
  :284-334  the combined g4dn.8xlarge label set: scheduled
  :335-394  the combined inf2.xlarge label set (accelerator labels): scheduled
  :395-408  vpc.amazonaws.com/pod-eni on a t3.large: not scheduled (t3 is not trunking-compatible)
  :622-639  pod-eni lands on a type advertising it
  :712-931  nvidia.com/gpu -> p3.8xlarge (2 nodes), habana.ai/gaudi -> dl1.24xlarge (1), aws.amazon.com/neuron ->
            inf2.24xlarge (2), trn1.2xlarge, neuroncore -> inf2.xlarge, vpc.amazonaws.com/efa -> dl1.24xlarge (1),
            amd.com/gpu -> g4ad.16xlarge (2)
  :1033-1049 local zones: the only subnet in test-zone-1a-local, a pod requiring that zone is scheduled
  :2245-2310 spot priced in test-zone-1a only: a spot m5.large NodePool pinned to test-zone-1b cannot launch; unpinned
            it launches
The Windows vpc.amazonaws.com/PrivateIPv4Address cases (:639-711) are in tests/test_reference_scenarios.py. Not
transcribed: the accelerator labels the fake puts on g4dn.8xlarge (:254-258, the suite's own TODO: a GPU type carries
Neuron labels only in the fake data; here the individual-label test finds them on inf2).
"""
import pytest

import scenarios
from kpamd.model import NodePool, PodShape

K = "karpenter.k8s.aws/"
OD_POOL = [("karpenter.sh/capacity-type", "In", ["on-demand"])]
BACKENDS = ["oracle", pytest.param("device", marks=pytest.mark.gpu)]


def _env(request, lib, backend, **kw):
    types = scenarios.fake_catalog(lib, **kw)
    ctx = request.getfixturevalue("ctx") if backend == "device" else None
    zones = [z for z, _ in kw["subnet_zones"]] if kw.get("subnet_zones") else None
    return scenarios.Env(backend, types, ctx=ctx, zones=zones)


def _provision(request, lib, backend, pools, shapes, counts, **kw):
    env = _env(request, lib, backend, **kw)
    try:
        return env.provision(pools, shapes, counts)
    finally:
        env.close()


def _pod(requests=None, node_selector=None, required=None):
    r = {"pods": 1000}
    r.update(requests or {})
    return PodShape(r, node_selector=dict(node_selector or {}), required_terms=[required] if required else [])


G4DN_LABELS = {
    "karpenter.sh/nodepool": "default",
    "topology.kubernetes.io/region": "us-east-1",
    "topology.kubernetes.io/zone": "test-zone-1a",
    "node.kubernetes.io/instance-type": "g4dn.8xlarge",
    "kubernetes.io/os": "linux",
    "kubernetes.io/arch": "amd64",
    "karpenter.sh/capacity-type": "on-demand",
    K + "instance-hypervisor": "nitro",
    K + "instance-encryption-in-transit-supported": "true",
    K + "instance-category": "g",
    K + "instance-generation": "4",
    K + "instance-family": "g4dn",
    K + "instance-size": "8xlarge",
    K + "instance-cpu": "32",
    K + "instance-cpu-manufacturer": "intel",
    K + "instance-cpu-sustained-clock-speed-mhz": "2500",
    K + "instance-memory": "131072",
    K + "instance-ebs-bandwidth": "9500",
    K + "instance-network-bandwidth": "50000",
    K + "instance-gpu-name": "t4",
    K + "instance-gpu-manufacturer": "nvidia",
    K + "instance-gpu-count": "1",
    K + "instance-gpu-memory": "16384",
    K + "instance-local-nvme": "900",
    "topology.k8s.aws/zone-id": "tstz1-1a",
    # deprecated labels (karpv1.NormalizedLabels)
    "failure-domain.beta.kubernetes.io/region": "us-east-1",
    "failure-domain.beta.kubernetes.io/zone": "test-zone-1a",
    "beta.kubernetes.io/arch": "amd64",
    "beta.kubernetes.io/os": "linux",
    "beta.kubernetes.io/instance-type": "g4dn.8xlarge",
    "topology.ebs.csi.aws.com/zone": "test-zone-1a",
}
INF2_LABELS = dict(G4DN_LABELS, **{
    "node.kubernetes.io/instance-type": "inf2.xlarge", K + "instance-category": "inf", K + "instance-generation": "2",
    K + "instance-family": "inf2", K + "instance-size": "xlarge", K + "instance-cpu": "4",
    K + "instance-cpu-sustained-clock-speed-mhz": "3600", K + "instance-cpu-manufacturer": "amd",
    K + "instance-memory": "16384", K + "instance-ebs-bandwidth": "10000", K + "instance-network-bandwidth": "2083",
    K + "instance-accelerator-name": "inferentia2", K + "instance-accelerator-manufacturer": "aws",
    K + "instance-accelerator-count": "1", "beta.kubernetes.io/instance-type": "inf2.xlarge"})
for k in ("instance-gpu-name", "instance-gpu-manufacturer", "instance-gpu-count", "instance-gpu-memory",
          "instance-local-nvme"):
    del INF2_LABELS[K + k]


def _solve_two_catalogues(request, lib, backend, shapes):
    """Solve with the suite's nodePool (AL2023 catalogue) and windowsNodePool (Windows 2022 catalogue)."""
    import kpamd
    from kpamd.model import Problem
    linux = scenarios.fake_catalog(lib)
    windows = scenarios.fake_catalog(lib, ami_family="Windows2022")
    pools = [NodePool("default", 0, 0, OD_POOL), NodePool("windows", 0, 1, OD_POOL)]
    s, c, u = scenarios.pods_of([1] * len(shapes))
    prob = Problem([linux, windows], pools, shapes, s, c, u, name="labels")
    if backend == "oracle":
        from oracle import pyoracle
        return pyoracle.solve(prob)
    ctx = request.getfixturevalue("ctx")
    cats = [kpamd.Catalog(ctx, linux, seqnum=1), kpamd.Catalog(ctx, windows, seqnum=1)]
    try:
        return kpamd.Scheduler(ctx, prob, catalogs=cats).solve()
    finally:
        for cat in cats:
            cat.close()


@pytest.mark.parametrize("backend", BACKENDS)
def test_individual_instance_type_labels(request, lib, backend):
    """:223-283: one pod per well-known label (the Windows build label through the Windows NodePool, the accelerator
    labels on inf2): every pod is scheduled."""
    sel = dict(G4DN_LABELS)
    sel.update({K + "instance-accelerator-name": "inferentia2", K + "instance-accelerator-manufacturer": "aws",
                K + "instance-accelerator-count": "1", "node.kubernetes.io/windows-build": "10.0.20348"})
    shapes = [_pod(node_selector={k: v}) for k, v in sel.items()]
    res = _solve_two_catalogues(request, lib, backend, shapes)
    unplaced = [list(sel)[i] for i, p in enumerate(res["placement"]) if p == -1]
    assert not unplaced, unplaced
    win = list(sel).index("node.kubernetes.io/windows-build")
    assert res["nodeclaims"][res["placement"][win]]["nodepool"] == 1


@pytest.mark.parametrize("backend", BACKENDS)
@pytest.mark.parametrize("labels,want", [(G4DN_LABELS, "g4dn.8xlarge"), (INF2_LABELS, "inf2.xlarge")])
def test_combined_instance_type_labels(request, lib, backend, labels, want):
    """:284-394: the whole label set of g4dn.8xlarge (and of inf2.xlarge, accelerator labels) on one pod."""
    nodes, pod_node = _provision(request, lib, backend, [NodePool("default", 0, 0, OD_POOL)],
                                 [_pod(node_selector=labels)], [1])
    assert pod_node == [0] and nodes[0]["type"] == want and nodes[0]["zone"] == "test-zone-1a"


@pytest.mark.parametrize("backend", BACKENDS)
def test_pod_eni_not_on_t3(request, lib, backend):
    """:395-408."""
    nodes, pod_node = _provision(request, lib, backend, [NodePool("default", 0, 0, OD_POOL)],
                                 [_pod({"vpc.amazonaws.com/pod-eni": 1000},
                                       node_selector={"node.kubernetes.io/instance-type": "t3.large"})], [1])
    assert pod_node == [None] and nodes == []


@pytest.mark.parametrize("backend", BACKENDS)
def test_pod_eni_on_a_trunking_type(request, lib, backend):
    """:622-639: the launched type advertises vpc.amazonaws.com/pod-eni (IsTrunkingCompatible)."""
    types = {t.name: t for t in scenarios.fake_catalog(lib)}
    nodes, pod_node = _provision(request, lib, backend, [NodePool("default", 0, 0, OD_POOL)],
                                 [_pod({"vpc.amazonaws.com/pod-eni": 1000})], [1])
    assert pod_node == [0] and types[nodes[0]["type"]].capacity["vpc.amazonaws.com/pod-eni"] > 0


def _only(name):
    return [("node.kubernetes.io/instance-type", "In", [name])]


@pytest.mark.parametrize("backend", BACKENDS)
@pytest.mark.parametrize("resource,amounts,pool_reqs,want,n_nodes", [
    ("nvidia.com/gpu", [1, 2, 4], OD_POOL, "p3.8xlarge", 2),       # :712-741
    ("habana.ai/gaudi", [1, 2, 4], OD_POOL, "dl1.24xlarge", 1),    # :742-770
    ("aws.amazon.com/neuron", [2, 2, 4], OD_POOL, "inf2.24xlarge", 2),  # :771-801
    ("aws.amazon.com/neuron", [1], _only("trn1.2xlarge"), "trn1.2xlarge", 1),       # :802-826
    ("aws.amazon.com/neuroncore", [2], _only("inf2.xlarge"), "inf2.xlarge", 1),     # :827-851
    ("vpc.amazonaws.com/efa", [1, 2], _only("dl1.24xlarge"), "dl1.24xlarge", 1),    # :852-880
    ("amd.com/gpu", [1, 2, 4], OD_POOL, "g4ad.16xlarge", 2),       # :881-910
])
def test_accelerator_requests(request, lib, backend, resource, amounts, pool_reqs, want, n_nodes):
    shapes = [_pod({resource: a * 1000}) for a in amounts]
    nodes, pod_node = _provision(request, lib, backend, [NodePool("default", 0, 0, pool_reqs)], shapes,
                                 [1] * len(shapes))
    assert None not in pod_node
    assert {nodes[i]["type"] for i in pod_node} == {want}
    assert len(set(pod_node)) == n_nodes


@pytest.mark.parametrize("backend", BACKENDS)
def test_local_zone(request, lib, backend):
    """:1033-1049: the EC2NodeClass's only subnet is in test-zone-1a-local (zone id tstz1-1alocal, where the fake
    offers m5.large); a pod requiring that zone is scheduled there."""
    nodes, pod_node = _provision(request, lib, backend, [NodePool("default", 0, 0, OD_POOL)],
                                 [_pod(required=[("topology.kubernetes.io/zone", "In", ["test-zone-1a-local"])])], [1],
                                 subnet_zones=[("test-zone-1a-local", "tstz1-1alocal")])
    assert pod_node == [0] and nodes[0]["zone"] == "test-zone-1a-local" and nodes[0]["type"] == "m5.large"


@pytest.mark.parametrize("backend", BACKENDS)
@pytest.mark.parametrize("pin_zone,scheduled", [(True, False), (False, True)])
def test_spot_zonal_availability(request, lib, backend, pin_zone, scheduled):
    """:2245-2310: spot prices exist for m5.large in test-zone-1a only (UpdateSpotPricing); a spot m5.large NodePool
    pinned to test-zone-1b has no available offering, unpinned it launches (in test-zone-1a, spot)."""
    reqs = [("karpenter.sh/capacity-type", "In", ["spot"])] + _only("m5.large")
    if pin_zone:
        reqs.append(("topology.kubernetes.io/zone", "In", ["test-zone-1b"]))
    nodes, pod_node = _provision(request, lib, backend, [NodePool("default", 0, 0, reqs)], [_pod()], [1],
                                 spot_history={("m5.large", "test-zone-1a"): 0.004})
    if not scheduled:
        assert pod_node == [None] and nodes == []
        return
    assert pod_node == [0] and nodes[0]["capacity_type"] == "spot" and nodes[0]["zone"] == "test-zone-1a"
