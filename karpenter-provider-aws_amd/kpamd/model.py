"""Python mirror of the reference objects on the hot path (names follow the reference).

  InstanceType / Offering   <- sigs.k8s.io/karpenter pkg/cloudprovider types, built by
                               R:pkg/providers/instancetype/types.go:123-155 and offering.go:101-150
  NodePool                  <- karpv1.NodePool (the fields NewNodeClaimTemplate reads)
  PodShape / pods           <- corev1.Pod fields the scheduler reads (requests, nodeSelector, node
                               affinity, tolerations); pods are (shape, creationTimestamp, uid)
  ExistingNode              <- state.StateNode as seen by upstream scheduling.ExistingNode

Requirements are lists of tuples (key, operator, values[, minValues]) exactly like
scheduling.NewRequirementWithFlexibility's arguments. Quantities are int milli-units.
"""
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

import numpy as np

Req = Tuple  # (key, op, [values], minValues|None)


@dataclass
class Offering:
    capacity_type: str
    zone: str
    zone_id: Optional[str]
    price: float
    available: bool
    reservation_id: Optional[str] = None
    reservation_type: Optional[str] = None
    reservation_capacity: int = 0


@dataclass
class InstanceType:
    name: str
    requirements: List[Req]
    capacity: Dict[str, int]
    overhead: Dict[str, int]
    offerings: List[Offering] = field(default_factory=list)

    def allocatable(self):
        out = dict(self.capacity)
        for k, v in self.overhead.items():
            if k in out:
                out[k] -= v
        return out


@dataclass
class NodePool:
    name: str
    weight: int = 0
    catalog: int = 0
    requirements: List[Req] = field(default_factory=list)
    labels: Dict[str, str] = field(default_factory=dict)
    taints: List[Tuple[str, str, str]] = field(default_factory=list)  # (key, value, effect)
    limits: Dict[str, int] = field(default_factory=dict)
    daemon_requests: Dict[str, int] = field(default_factory=dict)


@dataclass
class LabelSelector:
    """metav1.LabelSelector; match_expressions are (key, "In"|"NotIn"|"Exists"|"DoesNotExist", [values])."""
    match_labels: Dict[str, str] = field(default_factory=dict)
    match_expressions: List[Tuple[str, str, List[str]]] = field(default_factory=list)


@dataclass
class TopologySpread:
    """corev1.TopologySpreadConstraint. selector None = nil (selects nothing)."""
    topology_key: str
    max_skew: int = 1
    selector: Optional[LabelSelector] = None
    when_unsatisfiable: str = "DoNotSchedule"
    min_domains: Optional[int] = None
    node_affinity_policy: Optional[str] = None  # None = Honor
    node_taints_policy: Optional[str] = None    # None = Ignore


@dataclass
class PodAffinityTerm:
    """corev1.PodAffinityTerm (+ weight for a WeightedPodAffinityTerm). namespaces empty and no namespace_selector =
    the pod's namespace; a namespace_selector (LabelSelector; empty = every namespace) adds the problem's namespaces
    whose labels it matches (Problem.namespaces / Cluster.namespaces)."""
    topology_key: str
    selector: Optional[LabelSelector] = None
    namespaces: List[str] = field(default_factory=list)
    weight: int = 0
    namespace_selector: Optional[LabelSelector] = None


@dataclass
class PodShape:
    requests: Dict[str, int]
    node_selector: Dict[str, str] = field(default_factory=dict)
    required_terms: List[List[Req]] = field(default_factory=list)
    preferred_terms: List[Tuple[int, List[Req]]] = field(default_factory=list)
    tolerations: List[Tuple[str, str, str, str]] = field(default_factory=list)  # (key, op, value, effect)
    topology_spread: List[TopologySpread] = field(default_factory=list)
    labels: Dict[str, str] = field(default_factory=dict)
    namespace: str = "default"
    host_ports: List[Tuple[str, int, str]] = field(default_factory=list)  # GetHostPorts: (hostIP, hostPort, protocol)
    volume_requirements: List[Req] = field(default_factory=list)         # VolumeTopology.Inject input
    required_anti_affinity: List[PodAffinityTerm] = field(default_factory=list)
    preferred_anti_affinity: List[PodAffinityTerm] = field(default_factory=list)
    required_affinity: List[PodAffinityTerm] = field(default_factory=list)   # unsupported on the device path
    preferred_affinity: List[PodAffinityTerm] = field(default_factory=list)


@dataclass
class ExistingNode:
    name: str
    labels: Dict[str, str]
    available: Dict[str, int]
    requests: Dict[str, int] = field(default_factory=dict)
    taints: List[Tuple[str, str, str]] = field(default_factory=list)
    initialized: bool = True
    host_ports: List[Tuple[str, int, str]] = field(default_factory=list)  # HostPortUsage of its bound pods


@dataclass
class ClusterNode:
    """state.StateNode as disruption sees it: an existing node + its instance type + reschedulable pods."""
    node: ExistingNode
    catalog: int
    instance_type: int
    pods: List[int] = field(default_factory=list)   # indices into Cluster.pod_*
    deleting: bool = False                           # MarkedForDeletion: its pods join every simulation


@dataclass
class Cluster:
    catalogs: List[List[InstanceType]]
    nodepools: List[NodePool]
    nodes: List[ClusterNode]
    shapes: List[PodShape]
    pod_shape: np.ndarray
    pod_creation: np.ndarray
    pod_uid: np.ndarray
    candidates: List[int] = field(default_factory=list)  # disruption-cost order
    name: str = ""
    pending: List[int] = field(default_factory=list)  # provisionable pods bound to no node (indices into pod_*)
    spot_to_spot: bool = False                         # SpotToSpotConsolidation feature gate
    namespaces: Dict[str, Dict[str, str]] = field(default_factory=dict)  # cluster namespaces: name -> labels
    pod_uid_str: Optional[List[str]] = None  # metadata.uid per pod (kp_cluster.pod_uids): the exact Queue tie-break


@dataclass
class Problem:
    catalogs: List[List[InstanceType]]
    nodepools: List[NodePool]
    shapes: List[PodShape]
    pod_shape: np.ndarray           # uint32 [P]
    pod_creation: np.ndarray        # int64 [P]
    pod_uid: np.ndarray             # uint64 [P] (order-preserving UID key)
    existing: List[ExistingNode] = field(default_factory=list)
    max_instance_types: int = 100
    name: str = ""
    bound_pods: List[Tuple[str, Dict[str, str], int]] = field(default_factory=list)  # (namespace, labels, existing idx)
    namespaces: Dict[str, Dict[str, str]] = field(default_factory=dict)  # cluster namespaces: name -> labels
    reserved_offering_mode: int = 0  # 0 fallback (scheduler default), 1 strict (provisioner: DisableReservedCapacityFallback)
    pod_uid_str: Optional[List[str]] = None  # metadata.uid per pod (kp_solve_in.pod_uids): NewQueue's exact UID tie-break

    @property
    def n_pods(self):
        return int(len(self.pod_shape))


MI = 1 << 20
GI = 1 << 30


def cpu(m):
    return int(m)


def mem_mi(x):
    return int(x) * MI * 1000
