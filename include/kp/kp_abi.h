/*
 * kp_abi.h — C ABI of the MI355X-native Karpenter bin-packing hot path.
 *
 * This is the drop-in boundary a Go cgo shim binds. Every entry point
 * replaces one reference surface:
 *
 *   kp_catalog_upload      <- cloudprovider.CloudProvider.GetInstanceTypes result
 *                             (R:pkg/cloudprovider/cloudprovider.go:177-193 -> instancetype.DefaultProvider.List
 *                              R:pkg/providers/instancetype/instancetype.go:129-171 + offering.InjectOfferings
 *                              R:pkg/providers/instancetype/offering/offering.go:68-98), resident on device
 *                             until its seqnum changes (R:instancetype.go:225-237 cacheKey).
 *   kp_instance_type_resolve <- instancetype.NewInstanceType (R:pkg/providers/instancetype/types.go:123-155)
 *   kp_filter_compatible_available <- filter.CompatibleAvailableFilter
 *                             (R:pkg/providers/instance/filter/filter.go:39-64), batched: many
 *                             (requirements, requests) rows × one catalogue on the GPU.
 *   kp_launch_select       <- instance.DefaultProvider.Create's launch-side selection
 *                             (R:pkg/providers/instance/instance.go:117-125 Create -> filterInstanceTypes :242-270,
 *                              getCapacityType :504-518, checkODFallback :336-355, getOverrides :392-439), batched:
 *                             one row per NodeClaim being launched.
 *   kp_solve               <- upstream scheduling.Scheduler.Solve (sigs.k8s.io/karpenter
 *                             pkg/controllers/provisioning/scheduling/scheduler.go), reached from
 *                             R:pkg/providers/instancetype/suite_test.go:93,279 (NewProvisioner/ExpectProvisioned),
 *                             followed by Results.TruncateInstanceTypes(MaxInstanceTypes).
 *
 * Conventions
 *   - Every function returns int32: KP_OK (0) or a negative KP_E_* code. kp_last_error() gives text.
 *     KP_E_UNSUPPORTED means the input uses a feature the device path does not implement; the Go
 *     shim then runs the original CPU path.
 *   - Caller owns every input buffer; nothing is retained after a call returns (catalogues copy).
 *   - Quantities are int64 milli-units (resource.Quantity.MilliValue()): cpu "1" = 1000,
 *     memory "1Mi" = 1048576000. kp_resource_list.present marks which resources are set; it
 *     matters only for NodePool limits (R: upstream filterByRemainingResources iterates limit keys).
 *   - No C++ exceptions and no torch types cross this boundary.
 */
#ifndef KP_ABI_H
#define KP_ABI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KP_ABI_VERSION 12

enum kp_status {
  KP_OK = 0,
  KP_E_INVAL = -1,
  KP_E_NOMEM = -2,
  KP_E_DEVICE = -3,
  KP_E_UNSUPPORTED = -4,
  KP_E_NOTFOUND = -5,
  KP_E_CANCELED = -6, /* ABI v11: the caller's kp_cancel token was set while the call ran (ctx.Done) */
};

/* Resource axis, fixed (R:pkg/providers/instancetype/types.go:317-329,151-153; R:pkg/apis/v1/labels.go:69-81). */
enum kp_resource {
  KP_RES_CPU = 0,
  KP_RES_MEMORY = 1,
  KP_RES_EPHEMERAL_STORAGE = 2,
  KP_RES_PODS = 3,
  KP_RES_POD_ENI = 4,        /* vpc.amazonaws.com/pod-eni */
  KP_RES_EFA = 5,            /* vpc.amazonaws.com/efa */
  KP_RES_NVIDIA_GPU = 6,     /* nvidia.com/gpu */
  KP_RES_AMD_GPU = 7,        /* amd.com/gpu */
  KP_RES_NEURON = 8,         /* aws.amazon.com/neuron */
  KP_RES_NEURONCORE = 9,     /* aws.amazon.com/neuroncore */
  KP_RES_GAUDI = 10,         /* habana.ai/gaudi */
  KP_RES_PRIVATE_IPV4 = 11,  /* vpc.amazonaws.com/PrivateIPv4Address */
  KP_NUM_RESOURCES = 12
};

typedef struct kp_resource_list {
  int64_t milli[KP_NUM_RESOURCES];
  uint32_t present; /* bit r set <=> resource r present in the ResourceList */
  uint32_t reserved_;
} kp_resource_list;

/* corev1.NodeSelectorOperator */
enum kp_operator {
  KP_OP_IN = 0,
  KP_OP_NOT_IN = 1,
  KP_OP_EXISTS = 2,
  KP_OP_DOES_NOT_EXIST = 3,
  KP_OP_GT = 4,
  KP_OP_LT = 5
};

/* scheduling.NewRequirementWithFlexibility(key, op, minValues, values...) */
typedef struct kp_requirement {
  const char* key;
  int32_t op;          /* enum kp_operator */
  int32_t min_values;  /* < 0: nil */
  const char* const* values;
  uint32_t n_values;
  uint32_t reserved_;
} kp_requirement;

typedef struct kp_requirements {
  const kp_requirement* items;
  uint32_t n;
  uint32_t reserved_;
} kp_requirements;

typedef struct kp_label {
  const char* key;
  const char* value;
} kp_label;

enum kp_taint_effect {
  KP_EFFECT_ANY = 0, /* tolerations only: empty effect matches all */
  KP_EFFECT_NO_SCHEDULE = 1,
  KP_EFFECT_PREFER_NO_SCHEDULE = 2,
  KP_EFFECT_NO_EXECUTE = 3
};

typedef struct kp_taint {
  const char* key;
  const char* value;
  int32_t effect;
  int32_t reserved_;
} kp_taint;

enum kp_toleration_operator { KP_TOL_EQUAL = 0, KP_TOL_EXISTS = 1 };

typedef struct kp_toleration {
  const char* key;   /* "" or NULL: any key (requires KP_TOL_EXISTS) */
  const char* value;
  int32_t op;        /* enum kp_toleration_operator */
  int32_t effect;    /* enum kp_taint_effect; KP_EFFECT_ANY = all effects */
} kp_toleration;

/* cloudprovider.Offering as built by createOfferings (R:offering.go:115-147). */
typedef struct kp_offering {
  const char* capacity_type; /* karpenter.sh/capacity-type In {capacity_type} */
  const char* zone;          /* topology.kubernetes.io/zone In {zone}; NULL: no zone requirement */
  const char* zone_id;       /* topology.k8s.aws/zone-id In {zone_id}; NULL: no zone-id requirement */
  const char* reservation_id;   /* capacity-reservation-id In {id}; NULL: DoesNotExist (R:offering.go:136) */
  const char* reservation_type; /* capacity-reservation-type In {type}; NULL: DoesNotExist (R:offering.go:137) */
  double price;
  int32_t available;
  int32_t reservation_capacity; /* Offering.ReservationCapacity (R:offering.go:178): read by ReservedOfferingFilter.
                                   Filter and launch plans take reserved offerings (ABI v7), Solve plans too (ABI
                                   v9: NodeClaim.reserveOfferings against each reservation's capacity, see
                                   kp_solve_in.reserved_offering_mode), cluster plans too (ABI v10: every simulation
                                   reserves strictly, as SimulateScheduling's DisableReservedCapacityFallback) */
} kp_offering;

/* cloudprovider.InstanceType after InjectOfferings. */
typedef struct kp_instance_type {
  const char* name;
  kp_requirements requirements;
  kp_resource_list capacity;
  kp_resource_list overhead; /* Overhead.Total() = kube-reserved + system-reserved + eviction */
  const kp_offering* offerings;
  uint32_t n_offerings;
  uint32_t reserved_;
} kp_instance_type;

typedef struct kp_catalog_desc {
  const kp_instance_type* types;
  uint32_t n_types;
  uint32_t reserved_;
} kp_catalog_desc;

/* NodePool -> NodeClaimTemplate (upstream NewNodeClaimTemplate). Order does not matter: the solver
 * orders pools by weight desc then name asc (upstream nodepoolutils.OrderByWeight). */
typedef struct kp_nodepool {
  const char* name;
  int32_t weight;
  uint32_t catalog; /* index into kp_solve_in.catalogs / catalog_descs: GetInstanceTypes(nodePool) */
  kp_requirements requirements;  /* spec.template.spec.requirements (minValues allowed) */
  const kp_label* labels;        /* spec.template.metadata.labels (karpenter.sh/nodepool is added) */
  uint32_t n_labels;
  uint32_t n_taints;
  const kp_taint* taints;        /* spec.template.spec.taints */
  kp_resource_list limits;       /* remaining limits (spec.limits minus existing capacity); present = limited */
  kp_resource_list daemon_requests; /* daemonset overhead for this template */
} kp_nodepool;

typedef struct kp_preferred_term {
  int32_t weight;
  int32_t reserved_;
  kp_requirements preference;
} kp_preferred_term;

/* metav1.LabelSelector: matchLabels AND matchExpressions (In / NotIn / Exists / DoesNotExist). A nil selector
 * (is_nil != 0) selects nothing; an empty one selects everything (metav1.LabelSelectorAsSelector). */
enum kp_selector_operator { KP_SEL_IN = 0, KP_SEL_NOT_IN = 1, KP_SEL_EXISTS = 2, KP_SEL_DOES_NOT_EXIST = 3 };
typedef struct kp_selector_requirement {
  const char* key;
  int32_t op;        /* enum kp_selector_operator */
  uint32_t n_values;
  const char* const* values;
} kp_selector_requirement;
typedef struct kp_label_selector {
  const kp_label* match_labels;
  uint32_t n_match_labels;
  uint32_t n_match_expressions;
  const kp_selector_requirement* match_expressions;
  int32_t is_nil;
  int32_t reserved_;
} kp_label_selector;

/* corev1.TopologySpreadConstraint (upstream scheduling.TopologyGroup of TopologyTypeSpread). */
enum kp_when_unsatisfiable { KP_DO_NOT_SCHEDULE = 0, KP_SCHEDULE_ANYWAY = 1 };
enum kp_inclusion_policy { KP_POLICY_UNSET = 0, KP_POLICY_HONOR = 1, KP_POLICY_IGNORE = 2 };
typedef struct kp_topology_spread {
  const char* topology_key;
  int32_t max_skew;
  int32_t min_domains;          /* <= 0: nil */
  int32_t when_unsatisfiable;   /* ScheduleAnyway constraints are dropped one by one by Preferences.Relax */
  int32_t node_affinity_policy; /* UNSET = Honor */
  int32_t node_taints_policy;   /* UNSET = Ignore */
  int32_t reserved_;
  kp_label_selector selector;
} kp_topology_spread;

/* corev1.PodAffinityTerm (ABI v6): pod affinity / anti-affinity on the hostname or a label key (upstream
 * TopologyGroup of TopologyTypePodAffinity / TopologyTypePodAntiAffinity, and the inverse groups bound pods' required
 * anti-affinity terms create). The namespaces a term selects (upstream Topology.buildNamespaceList): no namespaces
 * and no namespaceSelector -> the pod's own namespace; else `namespaces` plus every namespace of
 * kp_solve_in.namespaces / kp_cluster.namespaces whose labels namespace_selector matches (ABI v8; an empty
 * selector matches them all). */
typedef struct kp_pod_affinity_term {
  const char* topology_key;
  kp_label_selector selector;
  const char* const* namespaces;  /* n_namespaces == 0 and no namespace selector: the pod's own namespace */
  uint32_t n_namespaces;
  int32_t weight;                 /* preferred terms: WeightedPodAffinityTerm.weight */
  int32_t has_namespace_selector; /* != 0: namespaceSelector set (namespace_selector) */
  int32_t reserved_;
  kp_label_selector namespace_selector;
} kp_pod_affinity_term;

/* A namespace of the cluster and its labels (ABI v8): what a namespaceSelector lists (corev1.NamespaceList). */
typedef struct kp_namespace {
  const char* name;
  const kp_label* labels;
  uint32_t n_labels;
  uint32_t reserved_;
} kp_namespace;

/* A container port with hostPort != 0, as upstream scheduling.GetHostPorts reads it (HostPortUsage). Two entries
 * conflict when protocol and port are equal and either IP is unspecified (0.0.0.0 / ::) or both IPs are equal. */
enum kp_protocol { KP_PROTO_TCP = 0, KP_PROTO_UDP = 1, KP_PROTO_SCTP = 2 };
typedef struct kp_host_port {
  const char* ip;     /* hostIP; NULL or "" = 0.0.0.0 (corev1 default) */
  int32_t port;       /* hostPort, 1..65535 */
  int32_t protocol;   /* enum kp_protocol; corev1 default TCP */
} kp_host_port;

/* A pod "shape": everything the scheduler reads from a pod except its identity. */
typedef struct kp_pod_shape {
  kp_resource_list requests;                 /* resources.RequestsForPods(pod) */
  const kp_label* node_selector;
  uint32_t n_node_selector;
  uint32_t n_required_terms;
  const kp_requirements* required_terms;     /* nodeAffinity required NodeSelectorTerms (ORed) */
  const kp_preferred_term* preferred_terms;  /* nodeAffinity preferred terms */
  uint32_t n_preferred_terms;
  uint32_t n_tolerations;
  const kp_toleration* tolerations;
  uint32_t n_topology_spread;
  uint32_t n_labels;
  const kp_topology_spread* topology_spread; /* spec.topologySpreadConstraints, in spec order */
  const char* namespace_;                    /* metadata.namespace (topology selectors are namespaced) */
  const kp_label* labels;                    /* metadata.labels (matched by topology selectors) */
  /* ABI v6 */
  const kp_host_port* host_ports;            /* GetHostPorts(pod): NodeClaim.Add / ExistingNode.CanAdd conflicts */
  uint32_t n_host_ports;
  uint32_t n_volume_requirements;
  /* VolumeTopology.Inject: the topology requirements of the pod's volumes (PV node affinity / StorageClass
   * allowedTopologies, resolved by the caller), appended to every required node-affinity term (one term is
   * created when the pod has none) before scheduling. */
  const kp_requirement* volume_requirements;
  /* podAntiAffinity and podAffinity required / preferred terms. Preferred terms act as required until
   * Preferences.Relax removes them, heaviest first (affinity terms before anti-affinity terms). */
  const kp_pod_affinity_term* required_anti_affinity;
  const kp_pod_affinity_term* preferred_anti_affinity;
  const kp_pod_affinity_term* required_affinity;
  const kp_pod_affinity_term* preferred_affinity;
  uint32_t n_required_anti_affinity;
  uint32_t n_preferred_anti_affinity;
  uint32_t n_required_affinity;
  uint32_t n_preferred_affinity;
} kp_pod_shape;

/* A pod already bound to a node of the cluster: what upstream Topology.countDomains lists (through the
 * kube client) to seed the domain counts of every topology group whose selector matches it. */
typedef struct kp_bound_pod {
  const char* namespace_;
  const kp_label* labels;
  uint32_t n_labels;
  uint32_t node;  /* index into kp_solve_in.existing */
  /* ABI v6: its required podAntiAffinity terms (Topology.updateInverseAntiAffinity: pods the selector selects
   * avoid the bound pod's domain) */
  const kp_pod_affinity_term* anti_affinity;
  uint32_t n_anti_affinity;
  uint32_t reserved_;
} kp_bound_pod;

typedef struct kp_pod {
  uint32_t shape;
  uint32_t reserved_;
  int64_t creation_unix;  /* metadata.creationTimestamp (1 s resolution, as in the API) */
  uint64_t uid_key;       /* order-preserving key of metadata.uid (string order of UIDs); ignored when the batch
                             passes the UIDs themselves (kp_solve_in.pod_uids / kp_cluster.pod_uids, ABI v10) */
} kp_pod;

/* In-flight or real node already in the cluster (upstream ExistingNode). */
typedef struct kp_existing_node {
  const char* name;
  const kp_label* labels;   /* node labels -> NewLabelRequirements */
  uint32_t n_labels;
  uint32_t n_taints;
  const kp_taint* taints;
  kp_resource_list available;  /* cachedAvailable: allocatable minus bound pods' requests */
  kp_resource_list requests;   /* initial requests: daemonset pods expected but not yet bound */
  int32_t initialized;
  int32_t reserved_;
  /* ABI v6: HostPortUsage of the pods bound to the node (in a kp_cluster: every bound pod, reschedulable or not) */
  const kp_host_port* host_ports;
  uint32_t n_host_ports;
  uint32_t reserved2_;
} kp_existing_node;

typedef struct kp_ctx kp_ctx;
typedef struct kp_catalog kp_catalog;
typedef struct kp_solve_result kp_solve_result;
typedef struct kp_solve_plan kp_solve_plan;

typedef struct kp_solve_in {
  const kp_catalog* const* catalogs;      /* device path: resident catalogue handles */
  const kp_catalog_desc* catalog_descs;   /* CPU oracle path: the same catalogues as plain arrays */
  uint32_t n_catalogs;
  uint32_t n_nodepools;
  const kp_nodepool* nodepools;
  const kp_existing_node* existing;
  uint32_t n_existing;
  uint32_t n_shapes;
  const kp_pod_shape* shapes;
  const kp_pod* pods;
  uint32_t n_pods;
  uint32_t max_instance_types;  /* scheduling.MaxInstanceTypes = 100; 0 = no truncation */
  const kp_bound_pod* bound_pods;  /* pods running on existing nodes (topology domain counts) */
  uint32_t n_bound_pods;
  uint32_t n_namespaces;           /* ABI v8: the cluster's namespaces (pod affinity namespaceSelector) */
  const kp_namespace* namespaces;
  /* ABI v9: capacity reservations inside the Solve (upstream NodeClaim.Add reserveOfferings + ReservationManager,
   * designed in R:designs/odcr.md:248-256): KP_RESERVED_FALLBACK (0, the scheduler's default) never fails an Add for
   * want of reservation capacity; KP_RESERVED_STRICT (1, the provisioner's DisableReservedCapacityFallback) fails an
   * Add whose NodeClaim is compatible with reserved offerings it cannot reserve, and does not relax the pod then. */
  uint32_t reserved_offering_mode;
  uint32_t reserved2_;
  /* ABI v10: metadata.uid of every pod (n_pods strings), or NULL. Given, the Queue's last tie-break (upstream NewQueue:
   * creationTimestamp, then UID) compares the UIDs as strings, exactly; kp_pod.uid_key is then ignored. */
  const char* const* pod_uids;
} kp_solve_in;

#define KP_RESERVED_FALLBACK 0
#define KP_RESERVED_STRICT 1

typedef struct kp_nodeclaim_info {
  uint32_t nodepool;        /* index into kp_solve_in.nodepools */
  uint32_t n_pods;
  uint32_t n_remaining;     /* InstanceTypeOptions before truncation */
  uint32_t n_options;       /* after OrderByPrice + Truncate */
  const uint32_t* pods;     /* pod indices in the order they were added */
  const uint32_t* options;  /* catalogue indices, cheapest-compatible-offering price asc then name asc */
  kp_resource_list requests;
  /* the NodeClaim's Requirements after FinalizeScheduling (hostname placeholder removed) as upstream
   * Requirements.NodeSelectorRequirements() renders them (Gt/Lt win over NotIn values): keys in byte order,
   * values sorted. Owned by the result. Topology spread narrows keys here (e.g. zone In {one zone}). */
  kp_requirements requirements;
} kp_nodeclaim_info;

typedef struct kp_solve_stats {
  double device_ms;         /* solve + finalize kernel time, HIP events on the solve stream */
  double host_ms;           /* kp_solve_run wall time (restore state, kernels, result copy-back) */
  double prepare_ms;        /* kp_solve_prepare wall time (compile + upload) */
  double solve_kernel_ms;   /* solve_kernel alone */
  double finalize_kernel_ms;
  uint64_t attempts;        /* NodeClaim.Add / ExistingNode.CanAdd evaluations */
  uint64_t bytes_algorithmic; /* bytes the device algorithm reads+writes */
  uint64_t pops;            /* queue pops */
  uint64_t phase_cycles[8]; /* diagnostic (KP_TIMING=1): per-phase shader cycles of the solve loop */
  uint64_t scanned;         /* diagnostic: in-flight NodeClaim positions the candidate pre-pass visited */
  uint64_t cursor_starts;   /* diagnostic: sum of first-fit cursor start positions (positions skipped) */
  uint64_t attempt_cycles[8]; /* diagnostic (KP_TIMING=1): wave 0's in-flight attempt split (merge, pod keys,
                                 Fits, offerings, minValues; [5] = attempts timed) */
  double catalog_ms;        /* part of prepare_ms spent compiling the catalogue half (dictionary, catalogue SoA,
                               NodeClaimTemplates); 0 when it came resident from the kp_ctx cache */
  uint32_t catalog_cached;  /* 1: the catalogue half was resident (same catalogues + NodePools; seqnums equal, or
                               re-applied in place: catalog_refreshed) */
  uint32_t catalog_refreshed; /* 1: the catalogues' seqnums had changed (ICE marks, prices) and the resident half's
                                 offerings and template options were re-applied in place, not recompiled */
  uint64_t fast_pods;       /* pods placed by solve_kernel's single-wave fast lane (no requirement merge) */
  uint64_t fast_cycles[6];  /* diagnostic (KP_TIMING=1): fast-lane cycles: pop, stage, sort, pre-pass, attempts, commit */
  uint64_t slow_sorts;      /* sort.Slice replays that ran the literal pdqsort (no stable-move shortcut) */
  uint64_t fast_bails[8];   /* pods the fast lane handed to the full path: ineligible (topology / existing nodes),
                               spilled sort arrays, long sort shift, long scan, requirement merge, minValues,
                               no in-flight NodeClaim took it, reserved */
  uint64_t reserved_offering_errors; /* ABI v9: pops whose addToNewNodeClaim failed on a ReservedOfferingError (strict
                                        mode; upstream Results.ReservedOfferingErrors: deferred, not relaxed) */
  uint64_t run_length_pods; /* ABI v11: pods the fast lane committed as part of a run (queue runs of one shape-level
                               onto one NodeClaim, committed k at a time: solve_kernel's run-length commit) */
  uint64_t order_chunks[5]; /* ABI v10, diagnostic: the chunked newNodeClaims order past the LDS sort capacity: peak
                               chunks, chunk splits, emptied chunks, directory (re)builds, final order mode (1 LDS,
                               2 chunked, 0 flat global) */
} kp_solve_stats;

/* ---- context ---------------------------------------------------------------------------- */
typedef struct kp_options {
  double vm_memory_overhead_percent; /* R:pkg/operator/options/options.go:53 default 0.075 */
  int32_t reserved_enis;             /* R:pkg/operator/options/options.go:55 default 0 */
  int32_t device;                    /* HIP device ordinal */
} kp_options;

int32_t kp_ctx_create(const kp_options* opts, kp_ctx** out);
/* ABI v12: test and measurement overrides of the library's kernel and path choices. Every field 0 (the state a context
 * is created in) is the production choice; no environment variable changes a path (a stray variable in the
 * controller's environment cannot pick another kernel). Cross-check tests and benchmarks set them per context,
 * between calls (not while a call on the context runs). */
typedef struct kp_overrides {
  int32_t fast_lane;           /* 0 auto (the run-length-commit variant where most queue neighbours share their shape),
                                  1 the plain variant, 2 the run-length-commit variant */
  int32_t sort_capacity;       /* 0: 8192 NodeClaims in the LDS order; n > 0: the chunked order past n NodeClaims */
  int32_t chunk_capacity;      /* 0: the chunked order's full directory; n > 0: at most n chunks (then the flat order);
                                  n < 0: no chunks (the flat order past sort_capacity) */
  int32_t template_table;      /* 0: Solve reads the template-options table; 1: it re-filters per template attempt */
  uint64_t table_shard_min;    /* 0: 1 << 20 (shape-level, template) pairs before a communicator shards the table */
  int32_t general_batch;       /* 0: batched general simulations (superset Solve); 1: every subset compiled alone */
  int32_t feasibility_kernel;  /* 0 by catalogue size (quad <= 1024 types, else bits); 1 the per-type global-gather
                                  kernel; 2 the one-row bits kernel at any size */
  int32_t feasibility_blocks;  /* 0: by row count; n > 0: n blocks */
  int32_t feasibility_temporal;/* 0: cheapest-price rows as non-temporal stores; 1: temporal stores */
  int32_t timing;              /* 1: solve_kernel phase probes (kp_solve_stats phase_cycles / fast_cycles) */
  int32_t host_timing;         /* 1: host compile / general-path phases on stderr */
} kp_overrides;
int32_t kp_ctx_set_overrides(kp_ctx* ctx, const kp_overrides* ov); /* NULL: back to all 0 */
int32_t kp_ctx_get_overrides(const kp_ctx* ctx, kp_overrides* out);
/* Drops the caller's reference. Catalogues, plans and communicators created on the context hold their own, so they
 * may be destroyed before or after it (a garbage collector finalizes in any order); the context's stream, events and
 * spare arena are freed with the last reference. */
void kp_ctx_destroy(kp_ctx* ctx);
const char* kp_last_error(void);
int32_t kp_abi_version(void);

/* ---- catalogue ---------------------------------------------------------------------------- */
/* ctx may be NULL for a host-only catalogue (kp_solve_validate); device entry points need a ctx one. */
int32_t kp_catalog_upload(kp_ctx* ctx, const kp_catalog_desc* desc, uint64_t seqnum, kp_catalog** out);
uint64_t kp_catalog_seqnum(const kp_catalog* cat);
uint32_t kp_catalog_size(const kp_catalog* cat);
void kp_catalog_destroy(kp_catalog* cat);

/* Offering availability / price change on a resident catalogue: the UnavailableOfferings.MarkUnavailable ->
 * SeqNum bump -> InjectOfferings rebuild of the reference (R:pkg/cache/unavailableofferings.go:66-92,
 * R:pkg/providers/instancetype/offering/offering.go:68-147, cache key R:offering.go:189-207) without re-parsing
 * the types. An update names an existing offering by (type index, capacity type, zone): every offering of that
 * type with that capacity type and zone (NULL zone: the offerings without a zone requirement) takes `available`
 * and, when price is not NaN, `price`. All-or-nothing: KP_E_INVAL (nothing changed) if any update names no
 * offering. On success the catalogue's seqnum becomes `seqnum`. */
typedef struct kp_offering_update {
  uint32_t type;              /* index into the uploaded types */
  int32_t available;          /* 0: ICE / unavailable, 1: available */
  const char* capacity_type;
  const char* zone;
  double price;               /* NaN: keep */
  /* ABI v7: capacity reservations (capacityreservation.Provider.MarkUnavailable / GetAvailableInstanceCount,
   * R:pkg/providers/instance/instance.go:470-484): a non-NULL reservation_id narrows the match to that
   * reservation's offerings; reservation_capacity >= 0 sets ReservationCapacity (-1: keep). */
  const char* reservation_id;
  int32_t reservation_capacity;
  int32_t reserved_;
} kp_offering_update;
int32_t kp_catalog_update_offerings(kp_catalog* cat, const kp_offering_update* updates, uint32_t n, uint64_t seqnum);

/* EC2 facts the reference reads from ec2types.InstanceTypeInfo (+ the static tables it joins). */
typedef struct kp_ec2_info {
  const char* name;
  int32_t vcpu;
  int32_t reserved0_;
  int64_t memory_mib;
  const char* arch;               /* "amd64" | "arm64" (already mapped via AWSToKubeArchitectures) */
  const char* hypervisor;
  int32_t encryption_in_transit;
  int32_t clock_mhz;              /* 0: no ProcessorInfo clock */
  const char* cpu_manufacturer;   /* "" : none */
  int64_t ebs_bandwidth_mbps;     /* 0: not EBS-optimized by default */
  int64_t network_bandwidth_mbps; /* 0: not in the bandwidth table */
  int64_t local_nvme_gb;          /* 0: none */
  const char* gpu_name;           /* "" : no GPU */
  const char* gpu_manufacturer;
  int32_t gpu_count;
  int32_t reserved1_;
  int64_t gpu_memory_mib;
  const char* accel_name;         /* "" : none */
  const char* accel_manufacturer;
  int32_t accel_count;
  int32_t neuron_devices;         /* NeuronInfo */
  int32_t neuron_cores_per_device;
  int32_t efa;
  int32_t max_enis;               /* NetworkCards[DefaultNetworkCardIndex].MaximumNetworkInterfaces */
  int32_t ipv4_per_eni;
  int32_t trunking;               /* Limits[name].IsTrunkingCompatible */
  int32_t branch_enis;            /* Limits[name].BranchInterface */
  int32_t in_limits_table;        /* name present in zz_generated.vpclimits.go */
  int32_t instance_storage_gb;    /* ABI v10: InstanceStorageInfo.TotalSizeInGB (any disk type); 0: local_nvme_gb */
} kp_ec2_info;

/* One kubelet eviction-signal value (memory.available / nodefs.available): a quantity or a percentage of the
 * node's capacity (R:pkg/providers/instancetype/types.go:571-598, computeEvictionSignal / mustParsePercentage). */
typedef struct kp_eviction_value {
  int32_t set;                   /* 0: the key is absent from the map */
  int32_t is_percent;            /* 1: "<p>%" (percent holds p; 100 disables the threshold) */
  double percent;
  int64_t milli;                 /* quantity in milli-units (resource.Quantity.MilliValue) when !is_percent */
} kp_eviction_value;

/* EC2NodeClass.spec.kubelet overrides (R:pkg/apis/v1/ec2nodeclass.go KubeletConfiguration). Resource maps carry
 * the keys the user set (present bits); eviction maps are nil unless has_* is set. */
typedef struct kp_kubelet {
  kp_resource_list kube_reserved;
  kp_resource_list system_reserved;
  int32_t has_eviction_hard;
  int32_t has_eviction_soft;
  kp_eviction_value hard_memory_available, hard_nodefs_available;
  kp_eviction_value soft_memory_available, soft_nodefs_available;
} kp_kubelet;

/* EC2NodeClass.spec.blockDeviceMappings entry (ABI v10): the fields ephemeralStorage reads
 * (R:pkg/providers/instancetype/types.go:349-385). */
typedef struct kp_block_device_mapping {
  const char* device_name;  /* deviceName; NULL: unset */
  int64_t volume_size;      /* ebs.volumeSize in bytes; < 0: nil */
  int32_t root_volume;      /* rootVolume */
  int32_t reserved_;
} kp_block_device_mapping;

/* EC2NodeClass.spec.instanceStorePolicy (ABI v10) */
#define KP_INSTANCE_STORE_NONE 0
#define KP_INSTANCE_STORE_RAID0 1

/* EC2NodeClass subset that changes results (AMI family, kubelet overrides, block devices). */
typedef struct kp_nodeclass {
  const char* region;
  const char* const* zones;      /* subnet zones (ZoneInfo) */
  const char* const* zone_ids;   /* parallel to zones; NULL entries allowed */
  uint32_t n_zones;
  int32_t max_pods;              /* < 0: nil */
  int32_t pods_per_core;         /* <= 0: nil */
  int32_t ami_family;            /* ABI v9: KP_AMI_* (EC2NodeClass.AMIFamily(); 0 = AL2023, the default alias) */
  const kp_kubelet* kubelet;     /* NULL: no kubelet block (defaults) */
  /* ABI v10: ephemeral-storage capacity (R:types.go:349-385): RAID0 -> the instance store's total size; else the
   * root-volume BDM's size, else (Custom) the last BDM's size or the 20Gi EBS default, else the BDM on the family's
   * ephemeral device; else the family's default ephemeral volume */
  const kp_block_device_mapping* block_device_mappings;
  uint32_t n_block_device_mappings;
  int32_t instance_store_policy; /* KP_INSTANCE_STORE_* */
} kp_nodeclass;

/* AMI families (R:pkg/providers/amifamily): their FeatureFlags (R:resolver.go:110-117, bottlerocket.go:126-132,
 * windows.go:101-108) and default ephemeral block device (al2023.go:98-108, al2.go:107-116, bottlerocket.go:95-112,
 * windows.go:88-99, custom.go:48-58) shape pods, kube-reserved memory, eviction and ephemeral storage. */
#define KP_AMI_AL2023 0
#define KP_AMI_AL2 1
#define KP_AMI_BOTTLEROCKET 2
#define KP_AMI_WINDOWS2019 3
#define KP_AMI_WINDOWS2022 4
#define KP_AMI_CUSTOM 5

/* instancetype.NewInstanceType capacity + Overhead.Total() (R:types.go:123-155, 313-598) for the nodeclass's AMI
 * family: Windows families add vpc.amazonaws.com/PrivateIPv4Address (IPv4 addresses per ENI - 1, types in the VPC
 * limits table, amd64 only: R:types.go:151-153, 477-484). The label half (computeRequirements, R:types.go:158-292)
 * is plain string marshalling and stays with the caller (kpamd/catalog.py mirrors it). */
int32_t kp_instance_type_resolve(const kp_options* opts, const kp_ec2_info* info, const kp_nodeclass* nc,
                                 kp_resource_list* capacity, kp_resource_list* overhead);

/* The three InstanceTypeOverhead lists NewInstanceType builds (R:types.go:145-149): kubeReservedResources
 * (R:types.go:500-533, overrides win), systemReservedResources (R:types.go:494-498) and evictionThreshold
 * (R:types.go:535-564: defaults, then the max over evictionHard and evictionSoft — soft honoured for AL2023's
 * EvictionSoftEnabled — of each signal, assigned over the defaults). kp_instance_type_resolve's overhead is
 * their sum (Overhead.Total()). */
int32_t kp_instance_type_overhead(const kp_options* opts, const kp_ec2_info* info, const kp_nodeclass* nc,
                                  kp_resource_list* kube_reserved, kp_resource_list* system_reserved,
                                  kp_resource_list* eviction_threshold);

/* ---- feasibility (CompatibleAvailableFilter, batched) ------------------------------------- */
typedef struct kp_feasibility_query {
  kp_requirements requirements;
  kp_resource_list requests;
} kp_feasibility_query;

/* For each query q: bit t of out_mask[q*words + t/64] <=> instance type t is compatible, fits and has
 * a compatible available offering (R:filter.go:51-64; AllowUndefinedWellKnownLabels). out_cheapest
 * (optional, n_queries × n_types) = cheapest compatible available offering price, +inf if none.
 * words = (n_types + 63) / 64. */
int32_t kp_filter_compatible_available(kp_ctx* ctx, const kp_catalog* cat, const kp_feasibility_query* queries,
                                       uint32_t n_queries, uint64_t* out_mask, double* out_cheapest,
                                       kp_solve_stats* stats);

/* Same split into prepare (compile + upload the rows, resident) and run (one launch; copy-out only into
 * non-NULL buffers) so many runs — or a benchmark — reuse resident inputs. */
typedef struct kp_filter_plan kp_filter_plan;
int32_t kp_filter_prepare(kp_ctx* ctx, const kp_catalog* cat, const kp_feasibility_query* queries, uint32_t n_queries,
                          int32_t with_cheapest, kp_filter_plan** out);
int32_t kp_filter_run(kp_filter_plan* plan, uint64_t* out_mask, double* out_cheapest, kp_solve_stats* stats);
/* ABI v11, the compact result (prepare with with_cheapest = KP_FILTER_COMPACT): per query the mask and the set of
 * offering classes its requirements admit (out_classes[q], bit c = class c of kp_filter_class_prices), instead of n_types
 * prices. The cheapest compatible available offering price of type t for query q is then
 *   min over c in out_classes[q] of prices[c * n_types + t]   (+inf: none)
 * which equals kp_filter_run's out_cheapest bit for bit for every type, whether its mask bit is set or not (both are
 * the cheapest available offering among the query's compatible classes; the mask adds the type's requirements and Fits):
 * a class's price row is the cheapest available offering of the type in that class. kp_filter_class_prices copies the
 * plan's resident [C][n_types] table (C <= 64 classes) and its class count; the consumer reads it once per catalogue
 * seqnum, not per query, and a plan whose catalogue seqnum moved refuses it (KP_E_INVAL) until kp_filter_refresh. */
enum { KP_FILTER_MASK_ONLY = 0, KP_FILTER_CHEAPEST = 1, KP_FILTER_COMPACT = 2 };
int32_t kp_filter_run_compact(kp_filter_plan* plan, uint64_t* out_mask, uint64_t* out_classes, kp_solve_stats* stats);
int32_t kp_filter_class_prices(kp_filter_plan* plan, double* out, uint32_t capacity, uint32_t* n_classes);
void kp_filter_plan_destroy(kp_filter_plan* plan);
/* Re-apply the catalogue's current offerings to a prepared plan: only the offering section of the resident
 * catalogue (available-class masks, per-(type, class) prices; ~C*T*16 bytes) is rebuilt and copied to the
 * device, the rows stay resident. `cat` must be the catalogue the plan was prepared on (KP_E_INVAL otherwise). */
int32_t kp_filter_refresh(kp_filter_plan* plan, const kp_catalog* cat);

/* ---- launch-side selection (instance.DefaultProvider.Create) -------------------------------------
 * For each NodeClaim: filterInstanceTypes (R:pkg/providers/instance/instance.go:242-270) =
 *   CompatibleAvailableFilter (R:filter.go:39-64) -> CapacityReservationTypeFilter / CapacityBlockFilter /
 *   ReservedOfferingFilter (R:filter.go:66-274: they replace a type's offerings; offerings equal in every label form
 *   one class, so a replaced slice keeps whole classes) ->
 *   ExoticInstanceTypeFilter (R:filter.go:279-318) -> SpotInstanceFilter (R:filter.go:328-386), each filter that
 *   empties the set failing the launch with InsufficientCapacityError; then InstanceTypes.Truncate(reqs,
 *   max_types) = OrderByPrice + cut + SatisfiesMinValues (error -> CreateError "InstanceTypeFilteringFailed");
 * getCapacityType (R:instance.go:504-518): reserved, then spot, if the requirements allow it and some remaining
 *   type has an available compatible offering of it (in its replaced offering slice), else on-demand;
 * checkODFallback (R:instance.go:336-355): on-demand launch while flexible to spot with < 5 types (a warning);
 * getOverrides (R:instance.go:392-439): per remaining type (in truncated order) its available offerings compatible
 *   with the requirements narrowed to the chosen capacity type, in the type's offering order, whose zone has a
 *   subnet (subnet_zones stands for ZonalSubnetsForLaunch); launch-template grouping by AMI is AWS I/O, out of scope. */
typedef struct kp_launch_request {
  kp_requirements requirements;   /* NodeClaim.Spec.Requirements (minValues allowed) */
  kp_resource_list requests;      /* NodeClaim.Spec.Resources.Requests */
  const uint32_t* instance_types; /* the instance types Create receives: catalogue indices, any order */
  uint32_t n_instance_types;      /* <= 1024 on the device path */
  uint32_t reserved_;
} kp_launch_request;

enum kp_launch_status {
  KP_LAUNCH_OK = 0,
  KP_LAUNCH_INSUFFICIENT_CAPACITY = 1, /* a filter left no instance type (failed_filter says which) */
  KP_LAUNCH_MINVALUES = 2              /* Truncate: the cheapest max_types types do not satisfy minValues */
};
enum kp_launch_filter { KP_FILTER_COMPATIBLE_AVAILABLE = 0, KP_FILTER_EXOTIC = 4, KP_FILTER_SPOT = 5 };

typedef struct kp_launch_result {
  int32_t status;             /* enum kp_launch_status */
  int32_t capacity_type;      /* 0 on-demand, 1 spot, 2 reserved (KP_LAUNCH_OK only) */
  uint32_t n_types;           /* types written to out_types (after filters + Truncate) */
  uint32_t n_overrides;       /* overrides written to out_overrides */
  int32_t failed_filter;      /* enum kp_launch_filter when INSUFFICIENT_CAPACITY, else -1 */
  uint32_t n_compatible;      /* types kept by CompatibleAvailableFilter */
  uint32_t rejected_exotic;   /* types removed by ExoticInstanceTypeFilter */
  uint32_t rejected_spot;     /* types removed by SpotInstanceFilter */
  int32_t od_fallback_warning;/* checkODFallback would log its error */
  int32_t reservation_type;   /* capacity_type 2: getCapacityReservationType (R:instance.go:520-530), 0 default,
                                 1 capacity-block, -1 none; else -1 */
  uint32_t rejected_reservation; /* types removed by the three reservation filters */
  int32_t reserved_;
} kp_launch_result;

/* out_types: [n][max_types] catalogue indices in launch order; out_overrides: [n][max_types * n_subnet_zones]
 * entries (type_index << 8) | zone, zone = index into subnet_zones. max_types = 60 in the reference
  * (maxInstanceTypes, R:instance.go:60). */
int32_t kp_launch_select(kp_ctx* ctx, const kp_catalog* cat, const kp_launch_request* reqs, uint32_t n,
                         const char* const* subnet_zones, uint32_t n_subnet_zones, uint32_t max_types,
                         kp_launch_result* out, uint32_t* out_types, uint32_t* out_overrides, kp_solve_stats* stats);
typedef struct kp_launch_plan kp_launch_plan;
int32_t kp_launch_prepare(kp_ctx* ctx, const kp_catalog* cat, const kp_launch_request* reqs, uint32_t n,
                          const char* const* subnet_zones, uint32_t n_subnet_zones, uint32_t max_types,
                          kp_launch_plan** out);
int32_t kp_launch_run(kp_launch_plan* plan, kp_launch_result* out, uint32_t* out_types, uint32_t* out_overrides,
                      kp_solve_stats* stats);
/* ICE / price refresh of a prepared launch plan from its catalogue (see kp_filter_refresh). */
int32_t kp_launch_refresh(kp_launch_plan* plan, const kp_catalog* cat);
void kp_launch_plan_destroy(kp_launch_plan* plan);

/* ---- Solve -------------------------------------------------------------------------------- */
/* kp_solve = kp_solve_prepare + kp_solve_run + kp_solve_plan_destroy. prepare compiles the batch (string
 * dictionaries -> bitsets, catalogue SoA, NodeClaimTemplates, pod queue order) and uploads it; run
 * executes Solve on the resident inputs and may be repeated (state is restored on device each run). */
int32_t kp_solve(kp_ctx* ctx, const kp_solve_in* in, kp_solve_result** out);
/* Host-side compile of the batch only (no device, catalogues may come from kp_catalog_upload(NULL, ...)):
 * KP_OK when kp_solve would accept it, else the KP_E_UNSUPPORTED / KP_E_INVAL it would return. */
int32_t kp_solve_validate(const kp_solve_in* in);
int32_t kp_solve_prepare(kp_ctx* ctx, const kp_solve_in* in, kp_solve_plan** out);
/* kp_solve_prepare as a collective over a communicator (kp_comm_init; NULL = this process alone): the per-Solve
 * table of template options per (shape-level, NodePool template) — addToNewNodeClaim's Compatible + Add +
 * filterInstanceTypesByRequirements for a fresh NodeClaim, SURVEY §8e "feasibility precompute" — is computed in
 * shape-level row ranges, one per rank, and all-gathered (ncclAllGather over xGMI); solve_kernel then reads one
 * entry per template attempt instead of re-filtering the template's types. Every rank passes the same batch; each
 * can then run the Solve (replicas) or only the committing rank does. */
struct kp_comm;
int32_t kp_solve_prepare_comm(kp_ctx* ctx, const kp_solve_in* in, struct kp_comm* comm, kp_solve_plan** out);
int32_t kp_solve_run(kp_solve_plan* plan, kp_solve_result** out);
/* ABI v11: cancellation (upstream Solve observes ctx.Done() between pods; SURVEY §5 failure handling). A kp_cancel
 * is a flag in host-mapped memory that solve_kernel polls about every 1,024 Queue pops; kp_cancel_set is lock-free
 * and may be called from any thread while a call runs (the cgo shim calls it when ctx.Done() fires). A run that sees
 * it set stops placing pods and returns KP_E_CANCELED with no result; the plan stays usable (every run restores its
 * state). The token stays set until kp_cancel_reset. One token may serve many calls, one at a time. */
typedef struct kp_cancel kp_cancel;
int32_t kp_cancel_create(kp_ctx* ctx, kp_cancel** out);
int32_t kp_cancel_set(kp_cancel* c);
int32_t kp_cancel_reset(kp_cancel* c);
void kp_cancel_destroy(kp_cancel* c);
/* kp_solve_run / kp_solve with a cancellation token (NULL: not cancellable, as kp_solve_run). */
int32_t kp_solve_run_cancellable(kp_solve_plan* plan, kp_cancel* cancel, kp_solve_result** out);
int32_t kp_solve_cancellable(kp_ctx* ctx, const kp_solve_in* in, kp_cancel* cancel, kp_solve_result** out);
/* A prepared plan after kp_catalog_update_offerings (UnavailableOfferings.MarkUnavailable + SeqNum,
 * R:pkg/cache/unavailableofferings.go:66-92): re-applies the catalogues' current availability and prices to the
 * resident catalogue half (offering masks, class prices and subset minima, the NodeClaimTemplates' options) and the
 * plan's template-options table, in place. kp_solve_run refuses a plan whose catalogues changed until this ran.
 * KP_E_INVAL when the update changed which NodePools keep any instance type (prepare again). A new kp_solve on the
 * same catalogues does the same on its own (stats.catalog_refreshed). */
int32_t kp_solve_refresh(kp_solve_plan* plan);
void kp_solve_plan_destroy(kp_solve_plan* plan);
uint32_t kp_result_nodeclaim_count(const kp_solve_result* res);
/* out[p] for every input pod: >= 0 new NodeClaim index; -1 pod error; <= -2 existing node -(2+i) */
int32_t kp_result_pod_placements(const kp_solve_result* res, int32_t* out, uint32_t n_pods);
int32_t kp_result_nodeclaim(const kp_solve_result* res, uint32_t i, kp_nodeclaim_info* out);
int32_t kp_result_stats(const kp_solve_result* res, kp_solve_stats* out);
void kp_result_destroy(kp_solve_result* res);

/* ---- Disruption: batched consolidation simulations ---------------------------------------------
 * Cluster snapshot as the disruption controller sees it (state.Cluster nodes + their reschedulable pods),
 * and a batch of candidate subsets. For each subset S, kp_simulate_batch computes what upstream
 * computeConsolidation(S...) decides (docs R:website/content/en/preview/concepts/disruption.md:89-128):
 * SimulateScheduling = Solve(pending pods + pods of the deleting nodes + pods of S, existing = every node that is
 * neither in S nor deleting) + TruncateInstanceTypes(100), with the NodePools' remaining limits; a pod of S placed
 * on an uninitialized node is an error (pods of deleting nodes are exempt); not all non-pending pods scheduled ->
 * no-op; 0 NodeClaims -> delete; > 1 -> no-op; 1 -> replace if some option's worst launch price is below the
 * summed candidate price (and, for multi-node, filterOutSameType keeps one). Spot-to-spot (feature gate, default
 * off) -> no-op. Subsets must not name deleting nodes. */
typedef struct kp_cluster_node {
  kp_existing_node node;      /* labels, taints, available (allocatable - bound pods), requests, initialized */
  uint32_t catalog;           /* catalogue of its instance type */
  uint32_t instance_type;     /* index of its instance type in that catalogue */
  const uint32_t* pods;       /* reschedulable pods on this node: indices into kp_cluster.pods */
  uint32_t n_pods;
  uint32_t deleting;          /* MarkedForDeletion: never a destination; its pods join every simulation */
} kp_cluster_node;

typedef struct kp_cluster {
  const kp_catalog* const* catalogs;      /* device path */
  const kp_catalog_desc* catalog_descs;   /* CPU oracle path */
  uint32_t n_catalogs;
  uint32_t n_nodepools;
  const kp_nodepool* nodepools;
  const kp_cluster_node* nodes;
  uint32_t n_nodes;
  uint32_t n_shapes;
  const kp_pod_shape* shapes;
  const kp_pod* pods;
  uint32_t n_pods;
  uint32_t spot_to_spot;      /* SpotToSpotConsolidation feature gate (default off; 1: spot candidates may be replaced
                                 by cheaper spot capacity, R:website/content/en/preview/concepts/disruption.md:110-128) */
  const uint32_t* pending_pods;  /* provisionable pods not bound to any node (indices into pods): they join every
                                    simulation, but their own scheduling errors do not block a decision */
  uint32_t n_pending;
  uint32_t n_namespaces;         /* ABI v8: the cluster's namespaces (pod affinity namespaceSelector) */
  const kp_namespace* namespaces;
  const char* const* pod_uids;   /* ABI v10: metadata.uid of every pod, or NULL (see kp_solve_in.pod_uids) */
} kp_cluster;

enum kp_decision { KP_DECISION_NOOP = 0, KP_DECISION_DELETE = 1, KP_DECISION_REPLACE = 2 };

typedef struct kp_sim_result {
  int32_t decision;           /* enum kp_decision */
  uint32_t replacement_nodepool;
  double candidate_price;     /* getCandidatePrices: sum of each candidate's cheapest label-compatible offering */
  double replacement_price;   /* REPLACE: min worst-launch price over the remaining replacement options */
  double savings;             /* DELETE: candidate_price; REPLACE: candidate_price - replacement_price; else 0 */
  uint32_t n_options;         /* REPLACE: replacement options left after the price filters */
  uint32_t n_pods;            /* pods rescheduled by the simulation */
} kp_sim_result;

/* subsets in CSR form: subset i = nodes[offsets[i] .. offsets[i+1]) (indices into cluster->nodes), in
 * candidate order. multi_node != 0 applies MultiNodeConsolidation's filterOutSameType to replacements. */
int32_t kp_simulate_batch(kp_ctx* ctx, const kp_cluster* cluster, const uint32_t* offsets, const uint32_t* nodes,
                          uint32_t n_subsets, int32_t multi_node, kp_sim_result* out, kp_solve_stats* stats);

/* Same, split so that one cluster snapshot serves many batches (the disruption loop re-probes one
 * snapshot: SingleNodeConsolidation, MultiNodeConsolidation's binary search, the sweep). prepare
 * compiles and uploads the snapshot and precomputes, per pod shape, the existing nodes it can ever use
 * and its NodeClaimTemplate outcome; simulate runs one batch of subsets on the resident snapshot.
 * NodePool limits, pending pods, deleting nodes, spot-to-spot and host ports run in the batched kernels; topology
 * spread, pod (anti-)affinity and a pod NotIn/DoesNotExist requirement on a label key some node lacks take the general
 * path (each subset a whole device Solve). Returns KP_E_UNSUPPORTED (the Go path then runs) for > 65535 pods in one
 * subset. Catalogues holding capacity reservations take the general path too (ABI v10): every simulation's Solve reserves
 * offerings strictly (SimulateScheduling's DisableReservedCapacityFallback); a candidate in a reservation is priced by
 * its reserved offering (on-demand / 1e7, R:pkg/providers/instancetype/offering/offering.go:160-166).
 * The general path compiles the cluster once as a superset Solve (every node not being deleted existing, every pod
 * a simulation can queue in its pod list) and runs the subsets' Solves batched, one workgroup each; a subset that
 * would remove every owner of an inverse anti-affinity term (and every subset of a cluster whose superset compile is
 * unsupported, or with kp_overrides.general_batch = 1) is compiled on its own. stats (general path): phase_cycles[0] simulations
 * batched, phase_cycles[1] simulations compiled per subset, phase_cycles[2] batched solve_kernel launches. */
typedef struct kp_cluster_plan kp_cluster_plan;
int32_t kp_cluster_prepare(kp_ctx* ctx, const kp_cluster* cluster, kp_cluster_plan** out);
int32_t kp_cluster_simulate(kp_cluster_plan* plan, const uint32_t* offsets, const uint32_t* nodes, uint32_t n_subsets,
                            int32_t multi_node, kp_sim_result* out, kp_solve_stats* stats);
/* ABI v12: kp_cluster_simulate with a cancellation token (NULL: as kp_cluster_simulate). Upstream runs consolidation
 * under a timeout and counts the ones that expire (karpenter_voluntary_disruption_consolidation_timeouts_total,
 * R:website/content/en/preview/reference/metrics.md:186-187); the disruption shim sets the token when its context
 * expires. The batched kernel reads the flag between a wave's subsets, the general path before each launch and inside
 * each simulation's Solve (every ~1,024 pops): the call returns KP_E_CANCELED with no result within about one
 * simulation's time, and the plan stays usable. */
int32_t kp_cluster_simulate_cancellable(kp_cluster_plan* plan, kp_cancel* cancel, const uint32_t* offsets,
                                        const uint32_t* nodes, uint32_t n_subsets, int32_t multi_node, kp_sim_result* out,
                                        kp_solve_stats* stats);
/* kp_solve_refresh for a cluster snapshot: after kp_catalog_update_offerings the catalogues' availability and
 * prices, the templates' options and the candidates' prices are re-applied in place and the per shape-level template
 * outcomes recomputed; kp_cluster_simulate / kp_consolidate_argmin refuse the plan until then. */
int32_t kp_cluster_refresh(kp_cluster_plan* plan);
void kp_cluster_plan_destroy(kp_cluster_plan* plan);

/* ---- Multi-GPU consolidation: RCCL over xGMI -----------------------------------------------------------------
 * One rank per GPU (one process per GPU, or one thread per GPU/kp_ctx in a single process): rank 0 calls
 * kp_comm_unique_id and hands the 128 bytes to every rank out of band; each rank calls kp_comm_init on its own
 * kp_ctx (collective: it returns once all n_ranks joined). SURVEY §8e: the subsets of a sweep shard by contiguous
 * index range; the snapshot is replicated (each rank prepares its own kp_cluster_plan from the same kp_cluster). */
#define KP_COMM_ID_BYTES 128
typedef struct kp_comm kp_comm;
int32_t kp_comm_unique_id(uint8_t* id /* KP_COMM_ID_BYTES */);
int32_t kp_comm_init(kp_ctx* ctx, const uint8_t* id, int32_t n_ranks, int32_t rank, kp_comm** out);
/* Single-process multi-GPU (the Karpenter controller is one leader-elected process): one kp_ctx per GPU, created by
 * the caller, and one call that builds their n communicators at once (ncclCommInitAll; rank i = ctxs[i], distinct
 * GPUs). Each rank is then driven by its own OS thread (one goroutine per GPU, runtime.LockOSThread): every
 * collective entry point (kp_solve_prepare_comm, kp_consolidate_argmin) must be called by all n threads for the
 * same step. out: n communicators. No unique-id transport is needed. */
int32_t kp_comm_init_all(kp_ctx* const* ctxs, int32_t n, kp_comm** out);
/* A communicator whose exchange step is a caller-supplied host all-gather: fn(user, rank, send, recv, bytes) must
 * block until every rank contributed `bytes` and fill recv with n_ranks * bytes in rank order, returning 0 (non-zero:
 * the step fails with KP_E_DEVICE). For transports other than RCCL (a gRPC stream between controller replicas, Go
 * channels between goroutines, a test harness); the records exchanged are small (status words, 88-byte choices, and
 * the template-options table only when it is sharded). */
typedef int32_t (*kp_allgather_fn)(void* user, int32_t rank, const void* send, void* recv, size_t bytes);
int32_t kp_comm_init_host(kp_ctx* ctx, int32_t n_ranks, int32_t rank, kp_allgather_fn fn, void* user, kp_comm** out);
int32_t kp_comm_rank(const kp_comm* comm, int32_t* rank, int32_t* n_ranks);
void kp_comm_destroy(kp_comm* comm);
/* Collective steps never leave a peer waiting: a rank whose local part fails still takes part in the exchange with
 * a failure record (kp_choice.subset = KP_CHOICE_FAILED, counts[0] = its error code; a status word in
 * kp_solve_prepare_comm), and then every rank returns an error. */
#define KP_CHOICE_FAILED (-2)

typedef struct kp_choice {
  int64_t subset;         /* global subset index of the best decision; -1: every subset of every rank is a no-op */
  uint64_t counts[3];     /* no-op / delete / replace decisions over all ranks' subsets */
  uint64_t overflowed;    /* subsets whose pods overflowed the device queue (kp_consolidate_argmin then fails) */
  kp_sim_result result;   /* computeConsolidation(subset) (decision, prices, savings, ...) */
} kp_choice;

/* The consolidation sweep step of one rank: simulate this rank's subsets (global indices base_index + i), reduce them
 * on the device to the best non-no-op decision (max savings, ties to the lowest global subset index), then one
 * RCCL all-gather of the ranks' 80-byte records over xGMI; every rank returns the same choice. comm NULL: this GPU
 * alone (n_ranks = 1). out (optional, n_subsets entries): the per-subset results, as kp_cluster_simulate.
 * Replaces the multi-node sweep the reference runs serially on one CPU (disruption.md:89-128). */
int32_t kp_consolidate_argmin(kp_cluster_plan* plan, kp_comm* comm, const uint32_t* offsets, const uint32_t* nodes,
                              uint32_t n_subsets, uint64_t base_index, int32_t multi_node, kp_sim_result* out,
                              kp_choice* best, kp_solve_stats* stats);
/* ABI v12: the sweep step with a cancellation token (see kp_cluster_simulate_cancellable). A rank whose token fires
 * still takes part in the all-gather (a KP_CHOICE_FAILED record holding KP_E_CANCELED), so no peer waits; every rank
 * then returns an error. */
int32_t kp_consolidate_argmin_cancellable(kp_cluster_plan* plan, kp_comm* comm, kp_cancel* cancel,
                                          const uint32_t* offsets, const uint32_t* nodes, uint32_t n_subsets,
                                          uint64_t base_index, int32_t multi_node, kp_sim_result* out, kp_choice* best,
                                          kp_solve_stats* stats);
/* The reduction kp_consolidate_argmin applies to the gathered per-rank records (host-only; exposed for callers that
 * reduce over another transport, and for tests): counts are summed, the best record wins. */
int32_t kp_choice_reduce(const kp_choice* per_rank, uint32_t n, kp_choice* out);

#ifdef __cplusplus
}
#endif
#endif /* KP_ABI_H */
