"""a5: EC2NodeClass kubelet overrides (kubeReserved, systemReserved, evictionHard, evictionSoft) in the instance
type overhead, transcribed from the reference's Overhead known-answer tests on m5.xlarge
(R:pkg/providers/instancetype/suite_test.go:1050-1553, BeforeEach at :1053-1064; the eviction contexts set
VMMemoryOverheadPercent 0, :1176-1180). Each KAT runs on the product (kp_instance_type_overhead, libkp host code,
no GPU) and on the oracle restatement (kpo_instance_type_resolve); the product's kp_instance_type_resolve overhead
must equal the sum of the three lists (Overhead.Total()).

AMI families (ABI v9 kp_nodeclass.ami_family): Bottlerocket ignores evictionSoft (:1397-1430); max-pods and the
kube-reserved memory per family on t3.large, with maxPods 10 (:1626-1670) and with reservedENIs 1 (:1697-1744);
Windows sets pods to 110 when the family has no ENI-limited density (:979-1001)."""
import ctypes as C

import pytest

from kpamd import abi, catalog

GI, MI = 1 << 30, 1 << 20
SYS_KUBE = {"system_reserved": {"memory": "20Gi"}, "kube_reserved": {"memory": "10Gi"}}


def _info(arena, name="m5.xlarge"):
    rows = {r["name"]: r for r in catalog.load_ec2_table()}
    return catalog.ec2_info(arena, rows[name])


def _opts(vm_overhead):
    o = catalog.default_options()
    if vm_overhead is not None:
        o.vm_memory_overhead_percent = vm_overhead
    return o


def product(lib, kubelet_cfg, vm_overhead=None, family="AL2023", name="m5.xlarge", max_pods=None, reserved_enis=0):
    arena = abi.Arena()
    opts, info = _opts(vm_overhead), _info(arena, name)
    opts.reserved_enis = reserved_enis
    nc = catalog.nodeclass(arena, kubelet_cfg=kubelet_cfg, ami_family=family, max_pods=max_pods)
    kube, sys_, ev = abi.ResourceList(), abi.ResourceList(), abi.ResourceList()
    assert lib.kp_instance_type_overhead(C.byref(opts), C.byref(info), C.byref(nc), C.byref(kube), C.byref(sys_),
                                         C.byref(ev)) == 0
    cap, total = abi.ResourceList(), abi.ResourceList()
    assert lib.kp_instance_type_resolve(C.byref(opts), C.byref(info), C.byref(nc), C.byref(cap), C.byref(total)) == 0
    parts = [catalog.resource_dict(x) for x in (kube, sys_, ev)]
    summed = {}
    for p in parts:
        for k, v in p.items():
            summed[k] = summed.get(k, 0) + v
    assert catalog.resource_dict(total) == summed, "Overhead.Total() = kube + system + eviction"
    return parts, catalog.resource_dict(cap)


def oracle(kubelet_cfg, vm_overhead=None, family="AL2023", name="m5.xlarge", max_pods=None, reserved_enis=0):
    from oracle import pyoracle
    arena = abi.Arena()
    nc = catalog.nodeclass(arena, kubelet_cfg=kubelet_cfg, ami_family=family, max_pods=max_pods)
    opts = _opts(vm_overhead)
    opts.reserved_enis = reserved_enis
    cap, ovh = pyoracle.instance_type_resolve(opts, _info(arena, name), nc)
    return [catalog.resource_dict(x) for x in (ovh.kube_reserved, ovh.system_reserved, ovh.eviction_threshold)], \
        catalog.resource_dict(cap)


BACKENDS = ["product", "oracle"]


def run(backend, lib, cfg, vm_overhead=None, **kw):
    return product(lib, cfg, vm_overhead, **kw) if backend == "product" else oracle(cfg, vm_overhead, **kw)


def q(d, k):
    """Quantity.String() == "0" for a missing key; values in milli-units."""
    return d.get(k, 0)


@pytest.mark.parametrize("backend", BACKENDS)
def test_system_reserved_defaults(backend, lib):
    (_, sys_, _), _ = run(backend, lib, {})  # R:suite_test.go:1067-1087
    assert q(sys_, "cpu") == q(sys_, "memory") == q(sys_, "ephemeral-storage") == 0


@pytest.mark.parametrize("backend", BACKENDS)
def test_system_reserved_override(backend, lib):
    cfg = {"system_reserved": {"cpu": "2", "memory": "20Gi", "ephemeral-storage": "10Gi"}}  # :1089-1116
    (_, sys_, _), _ = run(backend, lib, cfg)
    assert (sys_["cpu"], sys_["memory"], sys_["ephemeral-storage"]) == (2000, 20 * GI * 1000, 10 * GI * 1000)


@pytest.mark.parametrize("backend", BACKENDS)
def test_kube_reserved_defaults(backend, lib):
    (kube, _, _), _ = run(backend, lib, {})  # :1119-1139 -> 80m, 893Mi, 1Gi
    assert (kube["cpu"], kube["memory"], kube["ephemeral-storage"]) == (80, 893 * MI * 1000, GI * 1000)


@pytest.mark.parametrize("backend", BACKENDS)
def test_kube_reserved_override(backend, lib):
    cfg = {"system_reserved": {"cpu": "1", "memory": "20Gi", "ephemeral-storage": "1Gi"},
           "kube_reserved": {"cpu": "2", "memory": "10Gi", "ephemeral-storage": "2Gi"}}  # :1141-1172
    (kube, _, _), _ = run(backend, lib, cfg)
    assert (kube["cpu"], kube["memory"], kube["ephemeral-storage"]) == (2000, 10 * GI * 1000, 2 * GI * 1000)


def _approx(ev, cap, frac):
    """BeNumerically("~", capacity.memory * frac, 10): within 10 bytes."""
    return abs(ev["memory"] / 1000 - cap["memory"] / 1000 * frac) <= 10


# (kubelet maps on top of SYS_KUBE, expected eviction memory: bytes, or ("pct", fraction of capacity))
EVICTION_KATS = [
    ("hard quantity :1182", {"eviction_hard": {"memory.available": "500Mi"}}, 500 * MI),
    ("hard percent :1212", {"eviction_hard": {"memory.available": "10%"}}, ("pct", 0.10)),
    ("hard 100% disables :1242", {"eviction_hard": {"memory.available": "100%"}}, 0),
    ("soft only, hard unset :1272", {"eviction_soft": {"memory.available": "50Mi"}}, 50 * MI),
    ("soft quantity :1304", {"eviction_soft": {"memory.available": "500Mi"}}, 500 * MI),
    ("hard 5% soft 10% :1334", {"eviction_hard": {"memory.available": "5%"},
                                "eviction_soft": {"memory.available": "10%"}}, ("pct", 0.10)),
    ("soft 100% disables :1367", {"eviction_soft": {"memory.available": "100%"}}, 0),
    ("greater of soft 3Gi hard 1Gi :1454", {"eviction_soft": {"memory.available": "3Gi"},
                                            "eviction_hard": {"memory.available": "1Gi"}}, 3 * GI),
    ("greater of soft 2% hard 5% :1487", {"eviction_soft": {"memory.available": "2%"},
                                          "eviction_hard": {"memory.available": "5%"}}, ("pct", 0.05)),
    ("mixed soft 10% hard 1Gi :1520", {"eviction_soft": {"memory.available": "10%"},
                                       "eviction_hard": {"memory.available": "1Gi"}}, ("pct", 0.10)),
]


@pytest.mark.parametrize("backend", BACKENDS)
@pytest.mark.parametrize("name,maps,want", EVICTION_KATS, ids=[k[0] for k in EVICTION_KATS])
def test_eviction_threshold(backend, name, maps, want, lib):
    cfg = dict(SYS_KUBE, **maps)
    (_, _, ev), cap = run(backend, lib, cfg, vm_overhead=0.0)
    if isinstance(want, tuple):
        assert _approx(ev, cap, want[1]), (ev["memory"], cap["memory"])
    else:
        assert ev["memory"] == want * 1000


@pytest.mark.parametrize("backend", BACKENDS)
def test_eviction_default(backend, lib):
    (_, _, ev), _ = run(backend, lib, {}, vm_overhead=0.0)  # :1432-1452: 0 cpu, 100Mi, ~2Gi storage
    assert q(ev, "cpu") == 0 and ev["memory"] == 100 * MI * 1000
    assert ev["ephemeral-storage"] == pytest.approx(2 * GI * 1000)


@pytest.mark.parametrize("backend", BACKENDS)
def test_nodefs_signal(backend, lib):
    """nodefs.available follows the same rule on the ephemeral-storage capacity (R:types.go:552-554)."""
    (_, _, ev), cap = run(backend, lib, {"eviction_hard": {"nodefs.available": "15%"}}, vm_overhead=0.0)
    assert ev["ephemeral-storage"] == -(-cap["ephemeral-storage"] // 1000 * 15 // 100) * 1000


def test_product_matches_oracle_over_catalogue(lib):
    """Every catalogue type under one kubelet block with all four maps: product == oracle, list by list."""
    from oracle import pyoracle
    cfg = {"kube_reserved": {"cpu": "250m", "memory": "1Gi"}, "system_reserved": {"cpu": "100m"},
           "eviction_hard": {"memory.available": "7.5%", "nodefs.available": "1Gi"},
           "eviction_soft": {"memory.available": "300Mi", "nodefs.available": "12%"}}
    arena = abi.Arena()
    opts = catalog.default_options()
    nc = catalog.nodeclass(arena, kubelet_cfg=cfg)
    for r in catalog.load_ec2_table():
        info = catalog.ec2_info(arena, r)
        lists = [abi.ResourceList() for _ in range(3)]
        assert lib.kp_instance_type_overhead(C.byref(opts), C.byref(info), C.byref(nc), *map(C.byref, lists)) == 0
        _, ovh = pyoracle.instance_type_resolve(opts, info, nc)
        want = (ovh.kube_reserved, ovh.system_reserved, ovh.eviction_threshold)
        assert [catalog.resource_dict(x) for x in lists] == [catalog.resource_dict(x) for x in want], r["name"]


def test_parse_quantity():
    assert catalog.parse_quantity("2") == 2000 and catalog.parse_quantity("80m") == 80
    assert catalog.parse_quantity("20Gi") == 20 * GI * 1000 and catalog.parse_quantity("1.5") == 1500
    assert catalog.parse_quantity("1G") == 10**12 and catalog.parse_quantity("500Mi") == 500 * MI * 1000


# ---- AMI families -------------------------------------------------------------------------------------------
@pytest.mark.parametrize("backend", BACKENDS)
def test_bottlerocket_ignores_eviction_soft(backend, lib):
    """R:suite_test.go:1397-1430: Bottlerocket's EvictionSoftEnabled is false, so evictionHard alone sets it."""
    cfg = dict(SYS_KUBE, eviction_hard={"memory.available": "1Gi"}, eviction_soft={"memory.available": "10Gi"})
    (_, _, ev), _ = run(backend, lib, cfg, family="Bottlerocket")
    assert q(ev, "memory") == 1 * GI * 1000
    (_, _, ev2), _ = run(backend, lib, cfg, family="AL2023")  # the default family takes the larger soft signal
    assert q(ev2, "memory") == 10 * GI * 1000


FAMILY_MAXPODS = [("AL2", 10, 640), ("AL2023", 10, 640), ("Bottlerocket", 10, 365), ("Windows2019", 10, 365),
                  ("Windows2022", 10, 365), ("Custom", 10, 640)]  # R:suite_test.go:1664-1669 (11 * pods + 255 Mi)
FAMILY_RESERVED_ENIS = [("AL2", 24, 640), ("AL2023", 24, 640), ("Bottlerocket", 24, 519), ("Windows2019", 110, 1465),
                        ("Windows2022", 110, 1465), ("Custom", 24, 640)]  # R:suite_test.go:1738-1743


@pytest.mark.parametrize("backend", BACKENDS)
@pytest.mark.parametrize("family,pods,mem_mi", FAMILY_MAXPODS)
def test_family_max_pods_and_kube_reserved_memory(backend, lib, family, pods, mem_mi):
    """t3.large (3 ENIs x 12 IPv4), kubelet maxPods 10: pods 10 everywhere; kube-reserved memory from the ENI-limited
    count (35) for the families with UsesENILimitedMemoryOverhead, from pods() otherwise (R:suite_test.go:1626-1670)."""
    (kube, _, _), cap = run(backend, lib, {}, family=family, name="t3.large", max_pods=10)
    assert q(cap, "pods") == pods * 1000
    assert q(kube, "memory") == mem_mi * MI * 1000


@pytest.mark.parametrize("backend", BACKENDS)
@pytest.mark.parametrize("family,pods,mem_mi", FAMILY_RESERVED_ENIS)
def test_family_reserved_enis(backend, lib, family, pods, mem_mi):
    """reservedENIs 1: (3 - 1) * (12 - 1) + 2 = 24 pods where ENI-limited density applies, 110 on Windows
    (R:suite_test.go:1697-1744)."""
    (kube, _, _), cap = run(backend, lib, {}, family=family, name="t3.large", reserved_enis=1)
    assert q(cap, "pods") == pods * 1000
    assert q(kube, "memory") == mem_mi * MI * 1000


@pytest.mark.parametrize("backend", BACKENDS)
def test_windows_pods_110_and_private_ipv4(backend, lib):
    """R:suite_test.go:979-1001: a Windows nodeclass without maxPods gives every type 110 pods; amd64 types in the VPC
    limits table get PrivateIPv4Address = IPv4 per interface - 1 (R:types.go:151-153, 477-484), 50Gi root volume."""
    for name in ("m5.xlarge", "t3.large", "c6g.large"):
        _, cap = run(backend, lib, {}, family="Windows2022", name=name)
        assert q(cap, "pods") == 110 * 1000
        rows = {r["name"]: r for r in catalog.load_ec2_table()}
        r = rows[name]
        want = (r["ipv4_per_eni"] - 1) * 1000 if r["arch"] == "amd64" and r["eni_source"] == "vpclimits" else 0
        assert q(cap, "vpc.amazonaws.com/PrivateIPv4Address") == want
        assert q(cap, "ephemeral-storage") == 50 * GI * 1000


def test_product_equals_oracle_every_family(lib):
    """Capacity and the three overhead lists, product == oracle, for every docs type and every AMI family."""
    rows = catalog.load_ec2_table()
    for family in abi.AMI_FAMILIES:
        for r in rows[::7]:
            assert product(lib, dict(SYS_KUBE, eviction_soft={"memory.available": "5%"}), family=family, name=r["name"]) == \
                oracle(dict(SYS_KUBE, eviction_soft={"memory.available": "5%"}), family=family, name=r["name"]), (family, r["name"])
