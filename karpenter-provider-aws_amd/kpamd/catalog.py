"""Instance-type catalogue: host-side mirror of the reference's instancetype + offering providers.

  load_ec2_table()         the committed EC2 facts (tools/extract_fixtures.py; data, not source)
  compute_requirements()   R:pkg/providers/instancetype/types.go:158-292 computeRequirements (AL2023)
  resolve()                R:types.go:123-155 NewInstanceType — capacity and Overhead.Total() are
                           computed behind the C ABI by kp_instance_type_resolve (libkp)
  create_offerings()       R:pkg/providers/instancetype/offering/offering.go:101-150 createOfferings
                           with pricing lookups R:pkg/providers/pricing/pricing.go:145-170

Synthetic pricing: on-demand from the static us-east-1 table; spot = OD × U(0.3, 0.7)
per (type, zone) from splitmix64(seed=20250704), in table order then zone order.
"""
from dataclasses import dataclass
import ctypes as C
import os
import re

from . import abi
from .model import InstanceType, Offering

DATA = os.path.join(abi.PKG_ROOT, "data", "ec2_instance_types.tsv")
ZONES = ["test-zone-1a", "test-zone-1b", "test-zone-1c"]          # R:pkg/fake/ec2api.go:480-505
ZONE_IDS = ["tstz1-1a", "tstz1-1b", "tstz1-1c"]
REGION = "us-east-1"
SPOT_SEED = 20250704

INSTANCE_TYPE_SCHEME = re.compile(r"(^[a-z]+)(\-[0-9]+tb)?([0-9]+).*\.")  # R:types.go:49
K = "karpenter.k8s.aws/"

_INT_COLS = {"vcpu", "memory_mib", "gpu_count", "accel_count", "neuron_devices", "neuron_cores_per_device", "efa",
             "max_enis", "ipv4_per_eni", "trunking", "branch_enis"}


def load_ec2_table(path=DATA):
    rows = []
    with open(path) as f:
        header = None
        for line in f:
            if line.startswith("#"):
                continue
            parts = line.rstrip("\n").split("\t")
            if header is None:
                header = parts
                continue
            r = dict(zip(header, parts))
            for c in _INT_COLS:
                r[c] = int(r[c])
            r["od_price"] = float(r["od_price"])
            rows.append(r)
    return rows


class SplitMix64:
    def __init__(self, seed):
        self.s = seed & 0xFFFFFFFFFFFFFFFF

    def next(self):
        self.s = (self.s + 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF
        z = self.s
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
        return z ^ (z >> 31)

    def uniform(self):
        return (self.next() >> 11) * (1.0 / (1 << 53))


@dataclass
class CapacityReservation:
    """EC2NodeClass.status.capacityReservations entry (the fields createOfferings / computeRequirements read) plus the
    capacity reservation provider's available instance count (R:offering.go:165-170)."""
    id: str
    instance_type: str
    availability_zone: str
    reservation_type: str = "default"  # default | capacity-block
    available_count: int = 1


def compute_requirements(row, region=REGION, zones=ZONES, zone_ids=ZONE_IDS, offering_zones=None, reservations=(),
                         ami_family="AL2023"):
    """computeRequirements (R:types.go:158-292); reservations = the type's capacity reservations (reserved capacity
    type, reservation id / type In, R:types.go:172-174,223-232). Windows families: os In {windows} for amd64 types, no
    value otherwise (getOS, :294-302), windows-build In {the family's build} (:274-277)."""
    name = row["name"]
    offering_zones = zones if offering_zones is None else offering_zones
    available = [z for z in zones if z in set(offering_zones)]
    DNE = lambda k: (k, "DoesNotExist", [])
    reqs = {
        "node.kubernetes.io/instance-type": ("node.kubernetes.io/instance-type", "In", [name]),
        "kubernetes.io/arch": ("kubernetes.io/arch", "In", [row["arch"]]),
        "kubernetes.io/os": ("kubernetes.io/os", "In", ["linux"]) if ami_family not in abi.WINDOWS_BUILDS else
                            ("kubernetes.io/os", "In", ["windows"]) if row["arch"] == "amd64" else
                            ("kubernetes.io/os", "DoesNotExist", []),
        "topology.kubernetes.io/zone": ("topology.kubernetes.io/zone", "In", available),
        "topology.kubernetes.io/region": ("topology.kubernetes.io/region", "In", [region]),
        "node.kubernetes.io/windows-build": DNE("node.kubernetes.io/windows-build") if ami_family not in abi.WINDOWS_BUILDS
                                            else ("node.kubernetes.io/windows-build", "In", [abi.WINDOWS_BUILDS[ami_family]]),
        "karpenter.sh/capacity-type": ("karpenter.sh/capacity-type", "In",
                                       ["on-demand", "spot"] + (["reserved"] if reservations else [])),
        K + "instance-cpu": (K + "instance-cpu", "In", [str(row["vcpu"])]),
        K + "instance-memory": (K + "instance-memory", "In", [str(row["memory_mib"])]),
        K + "instance-hypervisor": (K + "instance-hypervisor", "In", [row["hypervisor"]]),
        K + "instance-encryption-in-transit-supported": (K + "instance-encryption-in-transit-supported", "In",
                                                         [row["encryption_in_transit"]]),
    }
    for k in ["instance-cpu-manufacturer", "instance-cpu-sustained-clock-speed-mhz", "instance-ebs-bandwidth",
              "instance-network-bandwidth", "instance-category", "instance-family", "instance-generation",
              "instance-local-nvme", "instance-size", "instance-gpu-name", "instance-gpu-manufacturer",
              "instance-gpu-count", "instance-gpu-memory", "instance-accelerator-name",
              "instance-accelerator-manufacturer", "instance-accelerator-count"]:
        reqs[K + k] = DNE(K + k)
    ids = [zid for z, zid in zip(zones, zone_ids) if z in set(available) and zid]
    if ids:
        reqs["topology.k8s.aws/zone-id"] = ("topology.k8s.aws/zone-id", "In", ids)
    if reservations:
        reqs[K + "capacity-reservation-id"] = (K + "capacity-reservation-id", "In", [cr.id for cr in reservations])
        reqs[K + "capacity-reservation-type"] = (K + "capacity-reservation-type", "In",
                                                 sorted({cr.reservation_type for cr in reservations}))
    else:
        reqs[K + "capacity-reservation-id"] = DNE(K + "capacity-reservation-id")
        reqs[K + "capacity-reservation-type"] = DNE(K + "capacity-reservation-type")

    def ins(k, v):
        reqs[K + k] = (K + k, "In", [v])

    m = INSTANCE_TYPE_SCHEME.search(name)
    if m:
        ins("instance-category", m.group(1))
        ins("instance-generation", m.group(3))
    parts = name.split(".")
    if len(parts) == 2:
        ins("instance-family", parts[0])
        ins("instance-size", parts[1])
    if row["local_nvme_gb"]:
        ins("instance-local-nvme", row["local_nvme_gb"])
    if row["network_bandwidth"]:
        ins("instance-network-bandwidth", row["network_bandwidth"])
    if row["gpu_name"]:
        ins("instance-gpu-name", row["gpu_name"])
        ins("instance-gpu-manufacturer", row["gpu_manufacturer"])
        ins("instance-gpu-count", str(row["gpu_count"]))
        ins("instance-gpu-memory", row["gpu_memory_mib"])
    if row["accel_name"]:
        ins("instance-accelerator-name", row["accel_name"])
        ins("instance-accelerator-manufacturer", row["accel_manufacturer"])
        ins("instance-accelerator-count", str(row["accel_count"]))
    ins("instance-cpu-manufacturer", row["cpu_manufacturer"])
    ins("instance-cpu-sustained-clock-speed-mhz", row["clock_mhz"])
    if row["ebs_bandwidth"]:
        ins("instance-ebs-bandwidth", row["ebs_bandwidth"])
    return list(reqs.values())


def ec2_info(arena, row):
    i = abi.EC2Info()
    s = arena.s
    i.name = s(row["name"])
    i.vcpu = row["vcpu"]
    i.memory_mib = row["memory_mib"]
    i.arch = s(row["arch"])
    i.hypervisor = s(row["hypervisor"])
    i.encryption_in_transit = 1 if row["encryption_in_transit"] == "true" else 0
    i.clock_mhz = int(row["clock_mhz"] or 0)
    i.cpu_manufacturer = s(row["cpu_manufacturer"])
    i.ebs_bandwidth_mbps = int(row["ebs_bandwidth"] or 0)
    i.network_bandwidth_mbps = int(row["network_bandwidth"] or 0)
    i.local_nvme_gb = int(row["local_nvme_gb"] or 0)
    # InstanceStorageInfo.TotalSizeInGB (RAID0 ephemeral storage, any disk type). The reference's offline tables only
    # carry it for NVMe instance stores (the instance-local-nvme label, R:types.go computeRequirements), so a row
    # without "instance_storage_gb" falls back to local_nvme_gb; a caller with the full EC2 answer passes both.
    i.instance_storage_gb = int(row.get("instance_storage_gb") or row["local_nvme_gb"] or 0)
    i.gpu_name = s(row["gpu_name"])
    i.gpu_manufacturer = s(row["gpu_manufacturer"])
    i.gpu_count = row["gpu_count"]
    i.gpu_memory_mib = int(row["gpu_memory_mib"] or 0)
    i.accel_name = s(row["accel_name"])
    i.accel_manufacturer = s(row["accel_manufacturer"])
    i.accel_count = row["accel_count"]
    i.neuron_devices = row["neuron_devices"]
    i.neuron_cores_per_device = row["neuron_cores_per_device"]
    i.efa = row["efa"]
    i.max_enis = row["max_enis"]
    i.ipv4_per_eni = row["ipv4_per_eni"]
    i.trunking = row["trunking"]
    i.branch_enis = row["branch_enis"]
    i.in_limits_table = 1 if row["eni_source"] == "vpclimits" else 0
    return i


_SUFFIX = {"": 1, "k": 10**3, "M": 10**6, "G": 10**9, "T": 10**12, "P": 10**15, "E": 10**18,
           "Ki": 2**10, "Mi": 2**20, "Gi": 2**30, "Ti": 2**40, "Pi": 2**50, "Ei": 2**60}


def parse_quantity(q):
    """resource.MustParse(q).MilliValue() for the plain forms kubelet maps use ("2", "80m", "1.5", "20Gi",
    "500Mi", "1G", "1e3"), exact (rational arithmetic, rounded up like MilliValue)."""
    from fractions import Fraction
    q = str(q).strip()
    if q.endswith("m") and not q.endswith("Mi"):
        return -(-Fraction(q[:-1]) // 1)
    for suf in sorted(_SUFFIX, key=len, reverse=True):
        if suf and q.endswith(suf):
            return -(-(Fraction(q[:-len(suf)]) * _SUFFIX[suf] * 1000) // 1)
    return -(-(Fraction(q) * 1000) // 1)


EVICTION_SIGNALS = {"memory.available": "memory_available", "nodefs.available": "nodefs_available"}


def _eviction_value(v):
    ev = abi.EvictionValue()
    ev.set = 1
    if str(v).endswith("%"):
        ev.is_percent, ev.percent = 1, float(str(v).strip("%"))  # strconv.ParseFloat(strings.Trim(v, "%"))
    else:
        ev.milli = parse_quantity(v)
    return ev


def kubelet(arena, kube_reserved=None, system_reserved=None, eviction_hard=None, eviction_soft=None):
    """EC2NodeClass.spec.kubelet resource/eviction maps -> kp_kubelet (string quantities as the CRD holds them).
    A None eviction map is nil; {} is an empty, non-nil map."""
    k = abi.Kubelet()
    k.kube_reserved = arena.resources({r: parse_quantity(v) for r, v in (kube_reserved or {}).items()})
    k.system_reserved = arena.resources({r: parse_quantity(v) for r, v in (system_reserved or {}).items()})
    for which, m in (("hard", eviction_hard), ("soft", eviction_soft)):
        if m is None:
            continue
        setattr(k, f"has_eviction_{which}", 1)
        for sig, v in m.items():
            if sig in EVICTION_SIGNALS:  # other signals (imagefs, pid) do not enter the overhead
                setattr(k, f"{which}_{EVICTION_SIGNALS[sig]}", _eviction_value(v))
    arena.keep.append(k)
    return k


def nodeclass(arena, zones=ZONES, zone_ids=ZONE_IDS, max_pods=None, pods_per_core=None, kubelet_cfg=None,
              ami_family="AL2023", block_device_mappings=None, instance_store_policy=None):
    """kp_nodeclass; kubelet_cfg: dict of kubelet(...) keyword arguments, or None for no kubelet block; ami_family:
    a key of abi.AMI_FAMILIES (EC2NodeClass.AMIFamily()); block_device_mappings: [(deviceName or None, volumeSize bytes
    or None, rootVolume)] (spec.blockDeviceMappings); instance_store_policy: None or "RAID0"."""
    nc = abi.NodeClass()
    nc.ami_family = abi.AMI_FAMILIES[ami_family]
    bdms = list(block_device_mappings or [])
    if bdms:
        nc.block_device_mappings = arena.arr(abi.BlockDeviceMapping, [
            abi.BlockDeviceMapping(arena.s(d), -1 if sz is None else int(sz), 1 if root else 0, 0) for d, sz, root in bdms])
    nc.n_block_device_mappings = len(bdms)
    nc.instance_store_policy = abi.INSTANCE_STORE_POLICIES[instance_store_policy]
    if kubelet_cfg is not None:
        nc.kubelet = C.pointer(kubelet(arena, **kubelet_cfg))
    nc.region = arena.s(REGION)
    nc.zones = arena.arr(C.c_char_p, [arena.s(z) for z in zones])
    nc.zone_ids = arena.arr(C.c_char_p, [arena.s(z) for z in zone_ids])
    nc.n_zones = len(zones)
    nc.max_pods = -1 if max_pods is None else max_pods
    nc.pods_per_core = 0 if pods_per_core is None else pods_per_core
    return nc


def resource_dict(rl):
    return {abi.RES_NAMES[i]: int(rl.milli[i]) for i in range(abi.NUM_RES) if rl.present & (1 << i)}


def create_offerings(row, reqs, spot_prices, zones=ZONES, zone_ids=ZONE_IDS, unavailable=frozenset(), reservations=()):
    """createOfferings (R:offering.go:101-186): zones × {on-demand, spot}, Available = !ICE ∧ hasPrice ∧
    zone∈itZones; then one reserved offering per capacity reservation of the type (price = OD / 1e7, 0 without an OD
    price; Available = available count != 0 ∧ zone∈itZones; ReservationCapacity = the count)."""
    it_zones = set(next(r for r in reqs if r[0] == "topology.kubernetes.io/zone")[2])
    zid = dict(zip(zones, zone_ids))
    out = []
    od = row["od_price"]
    for z in zones:
        for ct in ("on-demand", "spot"):
            if ct == "on-demand":
                price, has = (od, True) if od >= 0 else (0.0, False)
            else:
                price, has = (spot_prices[(row["name"], z)], True) if od >= 0 else (0.0, False)
            ice = (ct, row["name"], z) in unavailable or ct in unavailable or z in unavailable
            out.append(Offering(ct, z, zid.get(z), price, (not ice) and has and z in it_zones))
    for cr in reservations:
        out.append(Offering("reserved", cr.availability_zone, zid.get(cr.availability_zone),
                            od / 10_000_000.0 if od >= 0 else 0.0,
                            cr.available_count != 0 and cr.availability_zone in it_zones,
                            cr.id, cr.reservation_type, int(cr.available_count)))
    return out


def spot_price_table(rows, zones=ZONES, seed=SPOT_SEED):
    g = SplitMix64(seed)
    out = {}
    for r in rows:
        for z in zones:
            u = g.uniform()
            out[(r["name"], z)] = (r["od_price"] if r["od_price"] >= 0 else 0.0) * (0.3 + 0.4 * u)
    return out


def build_catalog(lib, rows=None, opts=None, max_pods=None, pods_per_core=None, zones=ZONES, zone_ids=ZONE_IDS,
                  unavailable=frozenset(), kubelet_cfg=None, capacity_reservations=(), ami_family="AL2023",
                  block_device_mappings=None, instance_store_policy=None):
    """GetInstanceTypes for one EC2NodeClass: NewInstanceType for every row, then InjectOfferings
    (capacity_reservations: the NodeClass's reservations, ReservedCapacity feature gate on)."""
    rows = load_ec2_table() if rows is None else rows
    arena = abi.Arena()
    opts = opts or default_options()
    nc = nodeclass(arena, zones, zone_ids, max_pods, pods_per_core, kubelet_cfg, ami_family, block_device_mappings,
                   instance_store_policy)
    spot = spot_price_table(rows, zones)
    out = []
    for r in rows:
        info = ec2_info(arena, r)
        cap, ovh = abi.ResourceList(), abi.ResourceList()
        rc = lib.kp_instance_type_resolve(C.byref(opts), C.byref(info), C.byref(nc), C.byref(cap), C.byref(ovh))
        if rc != 0:
            raise RuntimeError(f"kp_instance_type_resolve({r['name']}) = {rc}")
        crs = [cr for cr in capacity_reservations if cr.instance_type == r["name"]]  # R:types.go:117-119
        reqs = compute_requirements(r, zones=zones, zone_ids=zone_ids, reservations=crs, ami_family=ami_family)
        out.append(InstanceType(r["name"], reqs, resource_dict(cap), resource_dict(ovh),
                                create_offerings(r, reqs, spot, zones, zone_ids, unavailable, crs)))
    return out


def default_options(device=0):
    return abi.Options(0.075, 0, device)
