"""ctypes mirror of include/kp/kp_abi.h and the marshalling from Python model objects.

This is the Python analogue of the cgo shim a Go maintainer would add: it only
lays out C structs; every computation happens behind the C ABI.
"""
import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.dirname(HERE)

KP_OK, KP_E_INVAL, KP_E_NOMEM, KP_E_DEVICE, KP_E_UNSUPPORTED, KP_E_NOTFOUND, KP_E_CANCELED = 0, -1, -2, -3, -4, -5, -6
NUM_RES = 12
RES_NAMES = ["cpu", "memory", "ephemeral-storage", "pods", "vpc.amazonaws.com/pod-eni", "vpc.amazonaws.com/efa",
             "nvidia.com/gpu", "amd.com/gpu", "aws.amazon.com/neuron", "aws.amazon.com/neuroncore",
             "habana.ai/gaudi", "vpc.amazonaws.com/PrivateIPv4Address"]
RES_INDEX = {n: i for i, n in enumerate(RES_NAMES)}
OPS = {"In": 0, "NotIn": 1, "Exists": 2, "DoesNotExist": 3, "Gt": 4, "Lt": 5}
OP_NAMES = {v: k for k, v in OPS.items()}


def read_resources(r):
    """kp_resource_list -> {name: milli} (present entries only)"""
    return {RES_NAMES[i]: int(r.milli[i]) for i in range(NUM_RES) if (r.present >> i) & 1}


def read_requirements(r):
    """kp_requirements -> [(key, op, [values], minValues|None)]"""
    out = []
    for i in range(r.n):
        q = r.items[i]
        vals = [q.values[j].decode() for j in range(q.n_values)]
        out.append((q.key.decode(), OP_NAMES[q.op], vals, None if q.min_values < 0 else int(q.min_values)))
    return out


EFFECTS = {"": 0, "NoSchedule": 1, "PreferNoSchedule": 2, "NoExecute": 3}
TOL_OPS = {"Equal": 0, "": 0, "Exists": 1}


class ResourceList(C.Structure):
    _fields_ = [("milli", C.c_int64 * NUM_RES), ("present", C.c_uint32), ("reserved_", C.c_uint32)]


class Requirement(C.Structure):
    _fields_ = [("key", C.c_char_p), ("op", C.c_int32), ("min_values", C.c_int32),
                ("values", C.POINTER(C.c_char_p)), ("n_values", C.c_uint32), ("reserved_", C.c_uint32)]


class Requirements(C.Structure):
    _fields_ = [("items", C.POINTER(Requirement)), ("n", C.c_uint32), ("reserved_", C.c_uint32)]


class Label(C.Structure):
    _fields_ = [("key", C.c_char_p), ("value", C.c_char_p)]


class Taint(C.Structure):
    _fields_ = [("key", C.c_char_p), ("value", C.c_char_p), ("effect", C.c_int32), ("reserved_", C.c_int32)]


class Toleration(C.Structure):
    _fields_ = [("key", C.c_char_p), ("value", C.c_char_p), ("op", C.c_int32), ("effect", C.c_int32)]


class Offering(C.Structure):
    _fields_ = [("capacity_type", C.c_char_p), ("zone", C.c_char_p), ("zone_id", C.c_char_p),
                ("reservation_id", C.c_char_p), ("reservation_type", C.c_char_p),
                ("price", C.c_double), ("available", C.c_int32), ("reservation_capacity", C.c_int32)]


class OfferingUpdate(C.Structure):
    _fields_ = [("type", C.c_uint32), ("available", C.c_int32), ("capacity_type", C.c_char_p), ("zone", C.c_char_p),
                ("price", C.c_double), ("reservation_id", C.c_char_p), ("reservation_capacity", C.c_int32),
                ("reserved_", C.c_int32)]


class InstanceType(C.Structure):
    _fields_ = [("name", C.c_char_p), ("requirements", Requirements), ("capacity", ResourceList),
                ("overhead", ResourceList), ("offerings", C.POINTER(Offering)), ("n_offerings", C.c_uint32),
                ("reserved_", C.c_uint32)]


class CatalogDesc(C.Structure):
    _fields_ = [("types", C.POINTER(InstanceType)), ("n_types", C.c_uint32), ("reserved_", C.c_uint32)]


class NodePool(C.Structure):
    _fields_ = [("name", C.c_char_p), ("weight", C.c_int32), ("catalog", C.c_uint32),
                ("requirements", Requirements), ("labels", C.POINTER(Label)), ("n_labels", C.c_uint32),
                ("n_taints", C.c_uint32), ("taints", C.POINTER(Taint)), ("limits", ResourceList),
                ("daemon_requests", ResourceList)]


class PreferredTerm(C.Structure):
    _fields_ = [("weight", C.c_int32), ("reserved_", C.c_int32), ("preference", Requirements)]


SEL_OPS = {"In": 0, "NotIn": 1, "Exists": 2, "DoesNotExist": 3}
WHEN = {"DoNotSchedule": 0, "ScheduleAnyway": 1}
POLICY = {None: 0, "Honor": 1, "Ignore": 2}


class SelectorRequirement(C.Structure):
    _fields_ = [("key", C.c_char_p), ("op", C.c_int32), ("n_values", C.c_uint32), ("values", C.POINTER(C.c_char_p))]


class LabelSelector(C.Structure):
    _fields_ = [("match_labels", C.POINTER(Label)), ("n_match_labels", C.c_uint32),
                ("n_match_expressions", C.c_uint32), ("match_expressions", C.POINTER(SelectorRequirement)),
                ("is_nil", C.c_int32), ("reserved_", C.c_int32)]


class TopologySpread(C.Structure):
    _fields_ = [("topology_key", C.c_char_p), ("max_skew", C.c_int32), ("min_domains", C.c_int32),
                ("when_unsatisfiable", C.c_int32), ("node_affinity_policy", C.c_int32),
                ("node_taints_policy", C.c_int32), ("reserved_", C.c_int32), ("selector", LabelSelector)]


class PodAffinityTerm(C.Structure):
    _fields_ = [("topology_key", C.c_char_p), ("selector", LabelSelector), ("namespaces", C.POINTER(C.c_char_p)),
                ("n_namespaces", C.c_uint32), ("weight", C.c_int32), ("has_namespace_selector", C.c_int32),
                ("reserved_", C.c_int32), ("namespace_selector", LabelSelector)]


class Namespace(C.Structure):
    _fields_ = [("name", C.c_char_p), ("labels", C.POINTER(Label)), ("n_labels", C.c_uint32), ("reserved_", C.c_uint32)]


class HostPort(C.Structure):
    _fields_ = [("ip", C.c_char_p), ("port", C.c_int32), ("protocol", C.c_int32)]


PROTOCOLS = {"TCP": 0, "UDP": 1, "SCTP": 2, "": 0, None: 0}


class PodShape(C.Structure):
    _fields_ = [("requests", ResourceList), ("node_selector", C.POINTER(Label)), ("n_node_selector", C.c_uint32),
                ("n_required_terms", C.c_uint32), ("required_terms", C.POINTER(Requirements)),
                ("preferred_terms", C.POINTER(PreferredTerm)), ("n_preferred_terms", C.c_uint32),
                ("n_tolerations", C.c_uint32), ("tolerations", C.POINTER(Toleration)),
                ("n_topology_spread", C.c_uint32), ("n_labels", C.c_uint32),
                ("topology_spread", C.POINTER(TopologySpread)), ("namespace_", C.c_char_p),
                ("labels", C.POINTER(Label)), ("host_ports", C.POINTER(HostPort)), ("n_host_ports", C.c_uint32),
                ("n_volume_requirements", C.c_uint32), ("volume_requirements", C.POINTER(Requirement)),
                ("required_anti_affinity", C.POINTER(PodAffinityTerm)),
                ("preferred_anti_affinity", C.POINTER(PodAffinityTerm)),
                ("required_affinity", C.POINTER(PodAffinityTerm)), ("preferred_affinity", C.POINTER(PodAffinityTerm)),
                ("n_required_anti_affinity", C.c_uint32), ("n_preferred_anti_affinity", C.c_uint32),
                ("n_required_affinity", C.c_uint32), ("n_preferred_affinity", C.c_uint32)]


class BoundPod(C.Structure):
    _fields_ = [("namespace_", C.c_char_p), ("labels", C.POINTER(Label)), ("n_labels", C.c_uint32),
                ("node", C.c_uint32), ("anti_affinity", C.POINTER(PodAffinityTerm)), ("n_anti_affinity", C.c_uint32),
                ("reserved_", C.c_uint32)]


class Pod(C.Structure):
    _fields_ = [("shape", C.c_uint32), ("reserved_", C.c_uint32), ("creation_unix", C.c_int64), ("uid_key", C.c_uint64)]


class ExistingNode(C.Structure):
    _fields_ = [("name", C.c_char_p), ("labels", C.POINTER(Label)), ("n_labels", C.c_uint32),
                ("n_taints", C.c_uint32), ("taints", C.POINTER(Taint)), ("available", ResourceList),
                ("requests", ResourceList), ("initialized", C.c_int32), ("reserved_", C.c_int32),
                ("host_ports", C.POINTER(HostPort)), ("n_host_ports", C.c_uint32), ("reserved2_", C.c_uint32)]


class SolveIn(C.Structure):
    _fields_ = [("catalogs", C.POINTER(C.c_void_p)), ("catalog_descs", C.POINTER(CatalogDesc)),
                ("n_catalogs", C.c_uint32), ("n_nodepools", C.c_uint32), ("nodepools", C.POINTER(NodePool)),
                ("existing", C.POINTER(ExistingNode)), ("n_existing", C.c_uint32), ("n_shapes", C.c_uint32),
                ("shapes", C.POINTER(PodShape)), ("pods", C.POINTER(Pod)), ("n_pods", C.c_uint32),
                ("max_instance_types", C.c_uint32), ("bound_pods", C.POINTER(BoundPod)),
                ("n_bound_pods", C.c_uint32), ("n_namespaces", C.c_uint32), ("namespaces", C.POINTER(Namespace)),
                ("reserved_offering_mode", C.c_uint32), ("reserved2_", C.c_uint32),
                ("pod_uids", C.POINTER(C.c_char_p))]


class NodeClaimInfo(C.Structure):
    _fields_ = [("nodepool", C.c_uint32), ("n_pods", C.c_uint32), ("n_remaining", C.c_uint32),
                ("n_options", C.c_uint32), ("pods", C.POINTER(C.c_uint32)), ("options", C.POINTER(C.c_uint32)),
                ("requests", ResourceList), ("requirements", Requirements)]


class SolveStats(C.Structure):
    _fields_ = [("device_ms", C.c_double), ("host_ms", C.c_double), ("prepare_ms", C.c_double),
                ("solve_kernel_ms", C.c_double), ("finalize_kernel_ms", C.c_double), ("attempts", C.c_uint64),
                ("bytes_algorithmic", C.c_uint64), ("pops", C.c_uint64), ("phase_cycles", C.c_uint64 * 8),
                ("scanned", C.c_uint64), ("cursor_starts", C.c_uint64), ("attempt_cycles", C.c_uint64 * 8),
                ("catalog_ms", C.c_double), ("catalog_cached", C.c_uint32), ("catalog_refreshed", C.c_uint32),
                ("fast_pods", C.c_uint64), ("fast_cycles", C.c_uint64 * 6), ("slow_sorts", C.c_uint64),
                ("fast_bails", C.c_uint64 * 8), ("reserved_offering_errors", C.c_uint64), ("run_length_pods", C.c_uint64),
                ("order_chunks", C.c_uint64 * 5)]


class Options(C.Structure):
    _fields_ = [("vm_memory_overhead_percent", C.c_double), ("reserved_enis", C.c_int32), ("device", C.c_int32)]


class Overrides(C.Structure):
    """kp_overrides (ABI v12): test / measurement overrides of kernel and path choices; all 0 = production."""
    _fields_ = [("fast_lane", C.c_int32), ("sort_capacity", C.c_int32), ("chunk_capacity", C.c_int32),
                ("template_table", C.c_int32), ("table_shard_min", C.c_uint64), ("general_batch", C.c_int32),
                ("feasibility_kernel", C.c_int32), ("feasibility_blocks", C.c_int32),
                ("feasibility_temporal", C.c_int32), ("timing", C.c_int32), ("host_timing", C.c_int32)]


class EC2Info(C.Structure):
    _fields_ = [("name", C.c_char_p), ("vcpu", C.c_int32), ("reserved0_", C.c_int32), ("memory_mib", C.c_int64),
                ("arch", C.c_char_p), ("hypervisor", C.c_char_p), ("encryption_in_transit", C.c_int32),
                ("clock_mhz", C.c_int32), ("cpu_manufacturer", C.c_char_p), ("ebs_bandwidth_mbps", C.c_int64),
                ("network_bandwidth_mbps", C.c_int64), ("local_nvme_gb", C.c_int64), ("gpu_name", C.c_char_p),
                ("gpu_manufacturer", C.c_char_p), ("gpu_count", C.c_int32), ("reserved1_", C.c_int32),
                ("gpu_memory_mib", C.c_int64), ("accel_name", C.c_char_p), ("accel_manufacturer", C.c_char_p),
                ("accel_count", C.c_int32), ("neuron_devices", C.c_int32), ("neuron_cores_per_device", C.c_int32),
                ("efa", C.c_int32), ("max_enis", C.c_int32), ("ipv4_per_eni", C.c_int32), ("trunking", C.c_int32),
                ("branch_enis", C.c_int32), ("in_limits_table", C.c_int32), ("instance_storage_gb", C.c_int32)]


class EvictionValue(C.Structure):
    _fields_ = [("set", C.c_int32), ("is_percent", C.c_int32), ("percent", C.c_double), ("milli", C.c_int64)]


class Kubelet(C.Structure):
    _fields_ = [("kube_reserved", ResourceList), ("system_reserved", ResourceList),
                ("has_eviction_hard", C.c_int32), ("has_eviction_soft", C.c_int32),
                ("hard_memory_available", EvictionValue), ("hard_nodefs_available", EvictionValue),
                ("soft_memory_available", EvictionValue), ("soft_nodefs_available", EvictionValue)]


class BlockDeviceMapping(C.Structure):
    _fields_ = [("device_name", C.c_char_p), ("volume_size", C.c_int64), ("root_volume", C.c_int32),
                ("reserved_", C.c_int32)]


class NodeClass(C.Structure):
    _fields_ = [("region", C.c_char_p), ("zones", C.POINTER(C.c_char_p)), ("zone_ids", C.POINTER(C.c_char_p)),
                ("n_zones", C.c_uint32), ("max_pods", C.c_int32), ("pods_per_core", C.c_int32),
                ("ami_family", C.c_int32), ("kubelet", C.POINTER(Kubelet)),
                ("block_device_mappings", C.POINTER(BlockDeviceMapping)), ("n_block_device_mappings", C.c_uint32),
                ("instance_store_policy", C.c_int32)]


INSTANCE_STORE_POLICIES = {None: 0, "RAID0": 1}


AMI_FAMILIES = {"AL2023": 0, "AL2": 1, "Bottlerocket": 2, "Windows2019": 3, "Windows2022": 4, "Custom": 5}
WINDOWS_BUILDS = {"Windows2019": "10.0.17763", "Windows2022": "10.0.20348"}  # R:pkg/apis/v1/labels.go:111-112


class ClusterNode(C.Structure):
    _fields_ = [("node", ExistingNode), ("catalog", C.c_uint32), ("instance_type", C.c_uint32),
                ("pods", C.POINTER(C.c_uint32)), ("n_pods", C.c_uint32), ("deleting", C.c_uint32)]


class Cluster(C.Structure):
    _fields_ = [("catalogs", C.POINTER(C.c_void_p)), ("catalog_descs", C.POINTER(CatalogDesc)),
                ("n_catalogs", C.c_uint32), ("n_nodepools", C.c_uint32), ("nodepools", C.POINTER(NodePool)),
                ("nodes", C.POINTER(ClusterNode)), ("n_nodes", C.c_uint32), ("n_shapes", C.c_uint32),
                ("shapes", C.POINTER(PodShape)), ("pods", C.POINTER(Pod)), ("n_pods", C.c_uint32),
                ("spot_to_spot", C.c_uint32), ("pending_pods", C.POINTER(C.c_uint32)), ("n_pending", C.c_uint32),
                ("n_namespaces", C.c_uint32), ("namespaces", C.POINTER(Namespace)),
                ("pod_uids", C.POINTER(C.c_char_p))]


class SimResult(C.Structure):
    _fields_ = [("decision", C.c_int32), ("replacement_nodepool", C.c_uint32), ("candidate_price", C.c_double),
                ("replacement_price", C.c_double), ("savings", C.c_double), ("n_options", C.c_uint32),
                ("n_pods", C.c_uint32)]


class Choice(C.Structure):
    """kp_choice: the sweep's best decision over all ranks (kp_consolidate_argmin / kp_choice_reduce)."""
    _fields_ = [("subset", C.c_int64), ("counts", C.c_uint64 * 3), ("overflowed", C.c_uint64), ("result", SimResult)]


COMM_ID_BYTES = 128
CHOICE_FAILED = -2  # kp_choice.subset of a rank whose step failed
AllGatherFn = C.CFUNCTYPE(C.c_int32, C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p, C.c_size_t)


class FeasibilityQuery(C.Structure):
    _fields_ = [("requirements", Requirements), ("requests", ResourceList)]


class LaunchRequest(C.Structure):
    _fields_ = [("requirements", Requirements), ("requests", ResourceList),
                ("instance_types", C.POINTER(C.c_uint32)), ("n_instance_types", C.c_uint32), ("reserved_", C.c_uint32)]


class LaunchResult(C.Structure):
    _fields_ = [("status", C.c_int32), ("capacity_type", C.c_int32), ("n_types", C.c_uint32),
                ("n_overrides", C.c_uint32), ("failed_filter", C.c_int32), ("n_compatible", C.c_uint32),
                ("rejected_exotic", C.c_uint32), ("rejected_spot", C.c_uint32), ("od_fallback_warning", C.c_int32),
                ("reservation_type", C.c_int32), ("rejected_reservation", C.c_uint32), ("reserved_", C.c_int32)]


def launch_requests(arena, requests):
    """[(requirements, requests, [catalogue indices])] -> LaunchRequest array (buffers kept by the arena)."""
    out = []
    for reqs, res, types in requests:
        lst = arena.arr(C.c_uint32, [int(t) for t in types]) if len(types) else None
        out.append(LaunchRequest(arena.requirements(reqs), arena.resources(res), lst, len(types), 0))
    return arena.arr(LaunchRequest, out)


def launch_result_dict(r, types, ovr, zones):
    return {"status": int(r.status), "capacity_type": ("on-demand", "spot", "reserved")[int(r.capacity_type)],
            "types": [int(t) for t in types[:r.n_types]] if r.status == 0 else [],
            "overrides": [(int(o) >> 8, zones[int(o) & 0xFF]) for o in ovr[:r.n_overrides]] if r.status == 0 else [],
            "failed_filter": int(r.failed_filter), "n_compatible": int(r.n_compatible),
            "rejected_exotic": int(r.rejected_exotic), "rejected_spot": int(r.rejected_spot),
            "od_fallback_warning": bool(r.od_fallback_warning),
            "reservation_type": {0: "default", 1: "capacity-block"}.get(int(r.reservation_type)),
            "rejected_reservation": int(r.rejected_reservation)}


# ------------------------------------------------------------------------------------------------
# Marshalling: Python model objects (kpamd.model) -> ctypes, keeping every buffer alive on `self.keep`.
# ------------------------------------------------------------------------------------------------
class Arena:
    def __init__(self):
        self.keep = []
        self._str = {}

    def s(self, x):
        if x is None:
            return None
        b = self._str.get(x)
        if b is None:
            b = x.encode() if isinstance(x, str) else bytes(x)
            self._str[x] = b
        return b

    def arr(self, ctype, items):
        a = (ctype * max(1, len(items)))()
        for i, it in enumerate(items):
            a[i] = it
        self.keep.append(a)
        return a

    def uids(self, uids):
        """[metadata.uid] -> const char*[] (None: the batch passes no UIDs)"""
        if uids is None:
            return None
        return self.arr(C.c_char_p, [self.s(u) for u in uids])

    def resources(self, d):
        r = ResourceList()
        for k, v in (d or {}).items():
            i = RES_INDEX[k] if isinstance(k, str) else int(k)
            r.milli[i] = int(v)
            r.present |= 1 << i
        return r

    def requirement(self, req):
        key, op, values = req[0], req[1], list(req[2]) if len(req) > 2 and req[2] is not None else []
        min_values = req[3] if len(req) > 3 and req[3] is not None else -1
        vals = self.arr(C.c_char_p, [self.s(v) for v in values])
        return Requirement(self.s(key), OPS[op] if isinstance(op, str) else int(op), min_values, vals, len(values), 0)

    def requirements(self, reqs):
        items = self.arr(Requirement, [self.requirement(r) for r in (reqs or [])])
        return Requirements(items, len(reqs or []), 0)

    def labels(self, d):
        items = list((d or {}).items())
        return self.arr(Label, [Label(self.s(k), self.s(v)) for k, v in items]), len(items)

    def taints(self, ts):
        ts = ts or []
        return self.arr(Taint, [Taint(self.s(t[0]), self.s(t[1]), EFFECTS[t[2]], 0) for t in ts]), len(ts)

    def tolerations(self, ts):
        ts = ts or []
        out = []
        for t in ts:  # (key, operator, value, effect)
            out.append(Toleration(self.s(t[0] or ""), self.s(t[2] or ""), TOL_OPS[t[1]], EFFECTS[t[3] or ""]))
        return self.arr(Toleration, out), len(ts)

    def instance_types(self, its):
        out = []
        for it in its:
            ofs = self.arr(Offering, [Offering(self.s(o.capacity_type), self.s(o.zone), self.s(o.zone_id),
                                               self.s(getattr(o, "reservation_id", None)),
                                               self.s(getattr(o, "reservation_type", None)),
                                               float(o.price), 1 if o.available else 0,
                                               int(getattr(o, "reservation_capacity", 0))) for o in it.offerings])
            out.append(InstanceType(self.s(it.name), self.requirements(it.requirements), self.resources(it.capacity),
                                    self.resources(it.overhead), ofs, len(it.offerings), 0))
        return self.arr(InstanceType, out), len(its)

    def catalog_desc(self, its):
        a, n = self.instance_types(its)
        d = CatalogDesc(a, n, 0)
        self.keep.append(d)
        return d

    def nodepool(self, np, catalog_index):
        labels, nl = self.labels(np.labels)
        taints, nt = self.taints(np.taints)
        return NodePool(self.s(np.name), int(np.weight), catalog_index, self.requirements(np.requirements), labels, nl,
                        nt, taints, self.resources(np.limits), self.resources(np.daemon_requests))

    def shape(self, sh):
        ns, nns = self.labels(sh.node_selector)
        terms = self.arr(Requirements, [self.requirements(t) for t in sh.required_terms])
        prefs = self.arr(PreferredTerm, [PreferredTerm(int(w), 0, self.requirements(t)) for w, t in sh.preferred_terms])
        tols, ntol = self.tolerations(sh.tolerations)
        spreads = self.arr(TopologySpread, [self.spread(t) for t in sh.topology_spread])
        labels, nl = self.labels(sh.labels)
        hps, nhp = self.host_ports(getattr(sh, "host_ports", None))
        vol = list(getattr(sh, "volume_requirements", None) or [])
        vreqs = self.arr(Requirement, [self.requirement(r) for r in vol])
        ra, nra = self.affinity_terms(getattr(sh, "required_anti_affinity", None))
        pa, npa = self.affinity_terms(getattr(sh, "preferred_anti_affinity", None))
        rf, nrf = self.affinity_terms(getattr(sh, "required_affinity", None))
        pf, npf = self.affinity_terms(getattr(sh, "preferred_affinity", None))
        return PodShape(self.resources(sh.requests), ns, nns, len(sh.required_terms), terms, prefs,
                        len(sh.preferred_terms), ntol, tols, len(sh.topology_spread), nl, spreads,
                        self.s(sh.namespace), labels, hps, nhp, len(vol), vreqs, ra, pa, rf, pf, nra, npa, nrf, npf)

    def affinity_terms(self, terms):
        """[model.PodAffinityTerm] -> kp_pod_affinity_term[]."""
        terms = list(terms or [])
        out = []
        for t in terms:
            nss = self.arr(C.c_char_p, [self.s(n) for n in (t.namespaces or [])])
            nsel = t.namespace_selector
            out.append(PodAffinityTerm(self.s(t.topology_key), self.selector(t.selector), nss, len(t.namespaces or []),
                                       int(t.weight), 0 if nsel is None else 1, 0, self.selector(nsel)))
        return self.arr(PodAffinityTerm, out), len(terms)

    def namespaces(self, nss):
        """{name: labels} -> kp_namespace[] (sorted by name)."""
        out = []
        for name in sorted(nss or {}):
            lab, nl = self.labels(nss[name])
            out.append(Namespace(self.s(name), lab, nl, 0))
        return self.arr(Namespace, out), len(out)

    def host_ports(self, hps):
        """[(hostIP, hostPort, protocol)] -> kp_host_port[] (hostIP None/"" = 0.0.0.0, protocol None = TCP)."""
        hps = list(hps or [])
        return self.arr(HostPort, [HostPort(self.s(ip or ""), int(port), PROTOCOLS[proto]) for ip, port, proto in hps]), len(hps)

    def selector(self, sel):
        if sel is None:
            return LabelSelector(None, 0, 0, None, 1, 0)
        ml, nml = self.labels(sel.match_labels)
        exprs = []
        for key, op, values in sel.match_expressions:
            vals = self.arr(C.c_char_p, [self.s(v) for v in values])
            exprs.append(SelectorRequirement(self.s(key), SEL_OPS[op], len(values), vals))
        ex = self.arr(SelectorRequirement, exprs)
        return LabelSelector(ml, nml, len(exprs), ex, 0, 0)

    def spread(self, t):
        return TopologySpread(self.s(t.topology_key), int(t.max_skew), int(t.min_domains or 0),
                              WHEN[t.when_unsatisfiable], POLICY[t.node_affinity_policy],
                              POLICY[t.node_taints_policy], 0, self.selector(t.selector))

    def bound_pods(self, bps):
        out = []
        for bp in bps:  # (namespace, labels, existing idx[, required anti-affinity terms])
            ns, labels, node = bp[0], bp[1], bp[2]
            la, nl = self.labels(labels)
            aa, naa = self.affinity_terms(bp[3] if len(bp) > 3 else None)
            out.append(BoundPod(self.s(ns), la, nl, int(node), aa, naa, 0))
        return self.arr(BoundPod, out), len(bps)

    def existing_node(self, n, extra_ports=()):
        labels, nl = self.labels(n.labels)
        taints, nt = self.taints(n.taints)
        hps, nhp = self.host_ports(list(getattr(n, "host_ports", None) or []) + list(extra_ports))
        return ExistingNode(self.s(n.name), labels, nl, nt, taints, self.resources(n.available),
                            self.resources(n.requests), 1 if n.initialized else 0, 0, hps, nhp, 0)


def build_solve_in(arena, problem, catalog_handles=None):
    """problem: kpamd.model.Problem. catalog_handles: list of kp_catalog* (device path) or None."""
    descs = arena.arr(CatalogDesc, [arena.catalog_desc(c) for c in problem.catalogs]) if catalog_handles is None else None
    handles = arena.arr(C.c_void_p, catalog_handles) if catalog_handles is not None else None
    nps = arena.arr(NodePool, [arena.nodepool(np, np.catalog) for np in problem.nodepools])
    ex = arena.arr(ExistingNode, [arena.existing_node(n) for n in problem.existing])
    shapes = arena.arr(PodShape, [arena.shape(s) for s in problem.shapes])
    import numpy as np
    pods_np = np.zeros(len(problem.pod_shape), dtype=[("shape", "<u4"), ("r", "<u4"), ("c", "<i8"), ("u", "<u8")])
    pods_np["shape"] = problem.pod_shape
    pods_np["c"] = problem.pod_creation
    pods_np["u"] = problem.pod_uid
    arena.keep.append(pods_np)
    pods_ptr = pods_np.ctypes.data_as(C.POINTER(Pod))
    bps, nbp = arena.bound_pods(problem.bound_pods)
    nsa, nns = arena.namespaces(getattr(problem, "namespaces", None))
    si = SolveIn(handles, descs, len(problem.catalogs), len(problem.nodepools), nps, ex, len(problem.existing),
                 len(problem.shapes), shapes, pods_ptr, len(problem.pod_shape), problem.max_instance_types,
                 bps, nbp, nns, nsa if nns else None, getattr(problem, "reserved_offering_mode", 0), 0,
                 arena.uids(getattr(problem, "pod_uid_str", None)))
    arena.keep.append(si)
    return si


def _pods_array(arena, shape, creation, uid):
    import numpy as np
    pods_np = np.zeros(len(shape), dtype=[("shape", "<u4"), ("r", "<u4"), ("c", "<i8"), ("u", "<u8")])
    pods_np["shape"] = shape
    pods_np["c"] = creation
    pods_np["u"] = uid
    arena.keep.append(pods_np)
    return pods_np.ctypes.data_as(C.POINTER(Pod))


def build_cluster(arena, cl, catalog_handles=None):
    """kpamd.model.Cluster -> kp_cluster."""
    descs = arena.arr(CatalogDesc, [arena.catalog_desc(c) for c in cl.catalogs]) if catalog_handles is None else None
    handles = arena.arr(C.c_void_p, catalog_handles) if catalog_handles is not None else None
    nps = arena.arr(NodePool, [arena.nodepool(np, np.catalog) for np in cl.nodepools])
    nodes = []
    for n in cl.nodes:
        pods = arena.arr(C.c_uint32, list(n.pods))
        # the node's HostPortUsage: its own entries plus those of every pod bound to it (kp_cluster convention)
        used = [hp for p in n.pods for hp in (getattr(cl.shapes[int(cl.pod_shape[p])], "host_ports", None) or [])]
        nodes.append(ClusterNode(arena.existing_node(n.node, used), n.catalog, n.instance_type, pods, len(n.pods),
                                 1 if n.deleting else 0))
    nodes_a = arena.arr(ClusterNode, nodes)
    shapes = arena.arr(PodShape, [arena.shape(s) for s in cl.shapes])
    pending = list(cl.pending)
    nsa, nns = arena.namespaces(getattr(cl, "namespaces", None))
    c = Cluster(handles, descs, len(cl.catalogs), len(cl.nodepools), nps, nodes_a, len(cl.nodes), len(cl.shapes),
                shapes, _pods_array(arena, cl.pod_shape, cl.pod_creation, cl.pod_uid), len(cl.pod_shape),
                1 if cl.spot_to_spot else 0,
                arena.arr(C.c_uint32, pending) if pending else None, len(pending), nns, nsa if nns else None,
                arena.uids(getattr(cl, "pod_uid_str", None)))
    arena.keep.append(c)
    return c


SIM_DTYPE = None


def sim_dtype():
    import numpy as np
    global SIM_DTYPE
    if SIM_DTYPE is None:
        SIM_DTYPE = np.dtype([("decision", "<i4"), ("nodepool", "<u4"), ("candidate_price", "<f8"),
                              ("replacement_price", "<f8"), ("savings", "<f8"), ("n_options", "<u4"),
                              ("n_pods", "<u4")])
        assert SIM_DTYPE.itemsize == C.sizeof(SimResult)
    return SIM_DTYPE


def subsets_csr(arena, subsets):
    import numpy as np
    offs = np.zeros(len(subsets) + 1, dtype=np.uint32)
    offs[1:] = np.cumsum([len(s) for s in subsets])
    flat = np.concatenate([np.asarray(s, dtype=np.uint32) for s in subsets]) if subsets else np.zeros(1, np.uint32)
    arena.keep.extend([offs, flat])
    return offs.ctypes.data_as(C.POINTER(C.c_uint32)), flat.ctypes.data_as(C.POINTER(C.c_uint32))
