"""a4: ephemeral-storage capacity from the EC2NodeClass's blockDeviceMappings and instanceStorePolicy (ABI v10),
ephemeralStorage() R:pkg/providers/instancetype/types.go:349-385, on the product (kp_instance_type_resolve) and the
oracle restatement (kpo_instance_type_resolve).

Pinned by the reference's own tests:
  * the "Ephemeral Storage" context R:pkg/providers/instancetype/suite_test.go:2298-2382: a BDM without volumeSize on
    the family's device (/dev/xvda; /dev/xvdb for Bottlerocket) or a Custom AMI gives the EBS default, 20Gi capacity;
  * R:suite_test.go:932-954: a 5000Gi ephemeral-storage pod stays pending without instanceStorePolicy, and lands on
    m6idn.32xlarge with 7600G of ephemeral-storage capacity under RAID0 (fake 16-type catalogue, Solve + launch
    through tests/scenarios.py on the oracle here and on the device under -m gpu).
The remaining branches (a root volume's size, the device BDM's size, Custom's last BDM, Windows' 50Gi default, RAID0 on
a type without instance storage) follow the written control flow: parity with the oracle, not reference-pinned.
"""
import ctypes as C

import pytest

from kpamd import abi, catalog

GI = 1 << 30
EPH = "ephemeral-storage"


def _resolve(lib, name, family="AL2023", bdms=None, policy=None, row_update=None):
    rows = {r["name"]: r for r in catalog.load_ec2_table()}
    arena = abi.Arena()
    opts = catalog.default_options()
    info = catalog.ec2_info(arena, dict(rows[name], **(row_update or {})))
    nc = catalog.nodeclass(arena, ami_family=family, block_device_mappings=bdms, instance_store_policy=policy)
    cap, total = abi.ResourceList(), abi.ResourceList()
    assert lib.kp_instance_type_resolve(C.byref(opts), C.byref(info), C.byref(nc), C.byref(cap), C.byref(total)) == 0
    from oracle import pyoracle
    ocap, oovh = pyoracle.instance_type_resolve(opts, info, nc)
    prod = (catalog.resource_dict(cap), catalog.resource_dict(total))
    ev = catalog.resource_dict(oovh.eviction_threshold)
    osum = {}
    for part in (oovh.kube_reserved, oovh.system_reserved, oovh.eviction_threshold):
        for k, v in catalog.resource_dict(part).items():
            osum[k] = osum.get(k, 0) + v
    assert prod == (catalog.resource_dict(ocap), osum), "product == oracle"
    return prod[0][EPH] // 1000, ev[EPH] // 1000


XVDA_NO_SIZE = [("/dev/xvda", None, False)]  # the suite's BeforeEach (:2299-2309): snapshot id, no volumeSize


@pytest.mark.parametrize("family,bdms", [
    ("Custom", XVDA_NO_SIZE),                                   # :2311-2328
    ("AL2", XVDA_NO_SIZE),                                      # :2329-2343
    ("AL2023", XVDA_NO_SIZE),                                   # :2344-2360
    ("Bottlerocket", [("/dev/xvdb", None, False)]),             # :2361-2382
])
def test_ebs_default_when_volume_size_unset(lib, family, bdms):
    cap, ev = _resolve(lib, "m5.large", family, bdms)
    assert cap == 20 * GI
    assert ev == -(-cap * 10 // 100)  # the nodefs eviction default follows the same storage (ceil 10 %)


def test_raid0_uses_the_instance_store(lib):
    """R:suite_test.go:950: m6idn.32xlarge under RAID0 has 7600G of ephemeral storage (2 x 3800 GB NVMe)."""
    assert _resolve(lib, "m6idn.32xlarge", policy="RAID0")[0] == 7600 * 10**9
    assert _resolve(lib, "m6idn.32xlarge")[0] == 20 * GI  # no policy: the EBS default


@pytest.mark.parametrize("family,bdms,policy,want", [
    ("AL2023", [("/dev/xvdb", 80 * GI, False), ("/dev/xvdc", 60 * GI, True)], None, 60 * GI),  # the root volume's size
    ("AL2023", [("/dev/xvda", 100 * GI, False)], None, 100 * GI),          # the family device's size
    ("AL2023", [("/dev/xvdb", 100 * GI, False)], None, 20 * GI),           # another device: the family default
    ("AL2023", [("/dev/xvdb", None, True), ("/dev/xvda", 70 * GI, False)], None, 70 * GI),  # a sizeless root volume
    ("AL2023", [("/dev/xvda", None, True), ("/dev/xvda", 70 * GI, False)], None, 20 * GI),  # lo.Find: the first xvda
    ("Bottlerocket", [("/dev/xvda", 40 * GI, False)], None, 20 * GI),      # xvda is not Bottlerocket's data volume
    ("Bottlerocket", [("/dev/xvdb", 40 * GI, False)], None, 40 * GI),
    ("Windows2022", [], None, 50 * GI),                                    # /dev/sda1 50Gi
    ("Windows2019", [("/dev/sda1", 120 * GI, False)], None, 120 * GI),
    ("Custom", [("/dev/xvdb", 30 * GI, False), ("/dev/xvdc", 90 * GI, False)], None, 90 * GI),  # the last BDM
    ("Custom", [], None, 20 * GI),
    ("AL2023", [("/dev/xvda", 100 * GI, True)], "RAID0", 100 * GI),         # m5.large has no instance store
])
def test_ephemeral_storage_branches(lib, family, bdms, policy, want):
    assert _resolve(lib, "m5.large", family, bdms, policy)[0] == want


@pytest.mark.parametrize("backend", ["oracle", pytest.param("device", marks=pytest.mark.gpu)])
@pytest.mark.parametrize("policy", [None, "RAID0"])
def test_raid0_scenario(request, lib, backend, policy):
    """R:suite_test.go:932-954 on the fake catalogue (instancetype suite's on-demand NodePool): one pod requesting
    5000Gi of ephemeral storage stays pending without instanceStorePolicy; under RAID0 it launches on m6idn.32xlarge,
    whose ephemeral-storage capacity is 7600G."""
    import scenarios
    from kpamd.model import NodePool, PodShape
    types = scenarios.fake_catalog(lib, instance_store_policy=policy)
    ctx = request.getfixturevalue("ctx") if backend == "device" else None
    env = scenarios.Env(backend, types, ctx=ctx)
    try:
        pool = NodePool("default", 0, 0, [("karpenter.sh/capacity-type", "In", ["on-demand"])])
        nodes, pod_node = env.provision([pool], [PodShape({EPH: 5000 * GI * 1000, "pods": 1000})], [1])
    finally:
        env.close()
    if not policy:
        assert pod_node == [None] and nodes == []
        return
    assert pod_node == [0] and nodes[0]["type"] == "m6idn.32xlarge"
    assert next(t for t in types if t.name == "m6idn.32xlarge").capacity[EPH] == 7600 * 10**9 * 1000


def test_raid0_non_nvme_instance_store(lib):
    """RAID0 reads InstanceStorageInfo.TotalSizeInGB whatever the disk type. The reference's offline tables hold the
    total only for NVMe stores (instance-local-nvme), so the catalogue builder falls back to that; an EC2 answer for a
    non-NVMe store (no local-NVMe label, a total given) is used as is. NVMe: m6idn.32xlarge 7600G; a synthetic
    non-NVMe row: m5.large given a 6000 GB store and no NVMe label."""
    assert _resolve(lib, "m6idn.32xlarge", policy="RAID0", row_update={"instance_storage_gb": 7600})[0] == 7600 * 10**9
    non_nvme = {"instance_storage_gb": 6000, "local_nvme_gb": 0}
    assert _resolve(lib, "m5.large", policy="RAID0", row_update=non_nvme)[0] == 6000 * 10**9
    assert _resolve(lib, "m5.large", row_update=non_nvme)[0] == 20 * GI  # no policy: the EBS default
