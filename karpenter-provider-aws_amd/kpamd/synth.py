"""Synthetic workloads of BASELINE.json's configs and randomized parity scenarios.

All generators are deterministic in their seed. Pods are (shape, creationTimestamp, uid); every shape's
requests include pods=1 the way resources.RequestsForPods adds it.
"""
import numpy as np

from .catalog import ZONE_IDS, ZONES
from .model import Cluster, ClusterNode, ExistingNode, LabelSelector, NodePool, PodShape, Problem, TopologySpread

K = "karpenter.k8s.aws/"
MI = 1 << 20
CPU_GRID = [100, 250, 500, 1000, 2000, 4000]
MEM_GRID = [128, 256, 512, 1024, 2048, 4096, 8192]


def req_res(cpu_m, mem_mi, extra=None):
    r = {"cpu": int(cpu_m), "memory": int(mem_mi) * MI * 1000, "pods": 1000}
    if extra:
        r.update(extra)
    return r


def _pods(rng, n, n_shapes, weights=None):
    if weights is None:
        shape = rng.integers(0, n_shapes, size=n).astype(np.uint32)
    else:
        p = np.asarray(weights, dtype=np.float64)
        shape = rng.choice(n_shapes, size=n, p=p / p.sum()).astype(np.uint32)
    creation = (1_750_000_000 + rng.integers(0, 600, size=n)).astype(np.int64)
    uid = rng.integers(0, np.iinfo(np.int64).max, size=n, dtype=np.int64).astype(np.uint64)
    return shape, creation, uid


KWOK_POOL_REQS = [  # R:kwok/README.md:32-61
    ("kubernetes.io/arch", "In", ["amd64"]),
    ("kubernetes.io/os", "In", ["linux"]),
    ("karpenter.sh/capacity-type", "In", ["on-demand"]),
    (K + "instance-category", "In", ["c", "m", "r"]),
    (K + "instance-generation", "Gt", ["2"]),
]


def config1(catalog, n_pods=1000, seed=1):
    """1,000 pending pods (cpu/mem only) × full catalogue, the kwok README NodePool (limits cpu 1000)."""
    rng = np.random.default_rng(seed)
    shapes = [PodShape(req_res(c, m)) for c in CPU_GRID for m in MEM_GRID]
    s, c, u = _pods(rng, n_pods, len(shapes))
    np_ = NodePool("default", 0, 0, list(KWOK_POOL_REQS), limits={"cpu": 1000 * 1000})
    return Problem([catalog], [np_], shapes, s, c, u, name=f"config1-{n_pods}")


def config2(catalog, n_pods=50_000, seed=2, n_shapes=256, burst=False):
    """50k pods from 256 deployment shapes with mixed nodeSelector / node affinity / tolerations. burst: each
    deployment's pods are created within 2 s of its own start (ReplicaSet bursts) instead of uniformly over 600 s."""
    rng = np.random.default_rng(seed)
    shapes = []
    for i in range(n_shapes):
        cpu_m = int(rng.choice(CPU_GRID))
        mem = int(rng.choice(MEM_GRID))
        f = i / n_shapes
        sh = PodShape(req_res(cpu_m, mem))
        if f < 0.40:
            pass
        elif f < 0.60:
            sh.node_selector = {"topology.kubernetes.io/zone": ZONES[i % 3]}
        elif f < 0.75:
            if i % 2 == 0:
                sh.required_terms = [[(K + "instance-category", "In", ["c", "m", "r"])]]
            else:
                sh.required_terms = [[(K + "instance-cpu", "Gt", ["3"])]]
        elif f < 0.85:
            sh.required_terms = [[("kubernetes.io/arch", "NotIn", ["arm64"])]]
        else:
            sh.tolerations = [("dedicated", "Equal", "gpu", "NoSchedule")]
            sh.node_selector = {"karpenter.sh/nodepool": "dedicated"}
        shapes.append(sh)
    s, c, u = _pods(rng, n_pods, len(shapes))
    if burst:
        brng = np.random.default_rng(seed + 1000)
        start = brng.integers(0, 600, size=len(shapes))
        c = (1_750_000_000 + start[s] + brng.integers(0, 2, size=n_pods)).astype(np.int64)
    pools = [
        NodePool("general", 10, 0, [("kubernetes.io/os", "In", ["linux"]),
                                    ("karpenter.sh/capacity-type", "In", ["on-demand", "spot"]),
                                    (K + "instance-generation", "Gt", ["2"])]),
        NodePool("spot-compute", 5, 0, [("karpenter.sh/capacity-type", "In", ["spot"]),
                                        (K + "instance-category", "In", ["c", "m"])]),
        NodePool("dedicated", 1, 0, [("karpenter.sh/capacity-type", "In", ["on-demand"]),
                                     (K + "instance-generation", "Gt", ["4"])],
                 taints=[("dedicated", "gpu", "NoSchedule")]),
    ]
    return Problem([catalog], pools, shapes, s, c, u, name=f"config2-{n_pods}")


def config5(catalog, n_pods=1_000_000, seed=5, n_shapes=512, limit_div=1):
    """1M-pod burst over 20 weighted NodePools with cpu limits; 4 NVIDIA-GPU pools, 2 Neuron pools (tainted).
    limit_div > 1 divides every pool's cpu limit: the regime where the limits bind (38.7 % of 1M pods unschedulable)
    at a tenth of the pods (limit_div=10, 100k pods: 38.9 %)."""
    rng = np.random.default_rng(seed)
    pools = []
    for w in range(1, 21):
        name = f"pool-{w:02d}"
        limits = {"cpu": int(rng.integers(20_000, 200_000)) * 1000 // limit_div}  # ~2.2M cores: the burst spills by weight
        if w <= 4:
            pools.append(NodePool(name, w, 0, [(K + "instance-gpu-manufacturer", "In", ["nvidia"])],
                                  taints=[("nvidia.com/gpu", "true", "NoSchedule")], limits=limits))
        elif w <= 6:
            pools.append(NodePool(name, w, 0, [(K + "instance-accelerator-manufacturer", "In", ["aws"])],
                                  taints=[("aws.amazon.com/neuron", "true", "NoSchedule")], limits=limits))
        else:
            cats = [["c"], ["m"], ["r"], ["c", "m"], ["m", "r"], ["c", "m", "r"], ["t"]][w % 7]
            pools.append(NodePool(name, w, 0, [(K + "instance-category", "In", cats),
                                               ("karpenter.sh/capacity-type", "In", ["on-demand", "spot"])],
                                  limits=limits))
    shapes = []
    weights = []
    for i in range(n_shapes):
        cpu_m = int(rng.choice(CPU_GRID))
        mem = int(rng.choice(MEM_GRID))
        r = i % 16
        if r == 0:
            sh = PodShape(req_res(cpu_m, mem, {"nvidia.com/gpu": 1000 * int(rng.choice([1, 2, 4]))}),
                          tolerations=[("nvidia.com/gpu", "Exists", "", "NoSchedule")])
        elif r == 1:
            sh = PodShape(req_res(cpu_m, mem, {"aws.amazon.com/neuron": 1000}),
                          tolerations=[("aws.amazon.com/neuron", "Exists", "", "NoSchedule")])
        elif r < 6:
            sh = PodShape(req_res(cpu_m, mem), node_selector={"topology.kubernetes.io/zone": ZONES[i % 3]})
        else:
            sh = PodShape(req_res(cpu_m, mem))
        shapes.append(sh)
        weights.append(0.25 if r <= 1 else 1.0)
    s, c, u = _pods(rng, n_pods, len(shapes), weights)
    return Problem([catalog], pools, shapes, s, c, u, name=f"config5-{n_pods}")


# ------------------------------------------------------------------------------------------------
# config 3: topology spread onto existing nodes
# ------------------------------------------------------------------------------------------------
ZONE_KEY = "topology.kubernetes.io/zone"
HOST_KEY = "kubernetes.io/hostname"


def _type_named(catalog, name):
    for i, it in enumerate(catalog):
        if it.name == name:
            return i
    raise KeyError(name)


def config3(catalog, n_pods=100_000, seed=3, n_deployments=1000, n_existing=5000, prefill=0.3):
    """100k pods of 1,000 deployments, each spread over zones (maxSkew 1) and hostnames (maxSkew 1),
    DoNotSchedule, onto 5,000 existing m5/c5/r5 nodes (zones round-robin, ~30% of allocatable used by
    already-bound pods of the same deployments, which seed the topology counts) plus new NodeClaims."""
    rng = np.random.default_rng(seed)
    sizes = rng.integers(20, 181, size=n_deployments).astype(np.float64)
    counts = np.floor(sizes / sizes.sum() * n_pods).astype(np.int64)
    counts[: n_pods - int(counts.sum())] += 1
    shapes = []
    for j in range(n_deployments):
        app = {"app": f"dep-{j:04d}"}
        sel = LabelSelector(match_labels=dict(app))
        sh = PodShape(req_res(int(rng.choice([100, 250, 500, 1000, 2000])), int(rng.choice([128, 256, 512, 1024, 2048, 4096]))),
                      labels=dict(app), namespace=f"ns-{j % 8}",
                      topology_spread=[TopologySpread(ZONE_KEY, 1, sel), TopologySpread(HOST_KEY, 1, sel)])
        shapes.append(sh)
    pod_shape = np.repeat(np.arange(n_deployments, dtype=np.uint32), counts)
    rng.shuffle(pod_shape)
    n = len(pod_shape)
    creation = (1_750_000_000 + rng.integers(0, 600, size=n)).astype(np.int64)
    uid = rng.integers(0, np.iinfo(np.int64).max, size=n, dtype=np.int64).astype(np.uint64)
    pools = [NodePool("default", 10, 0, [("kubernetes.io/os", "In", ["linux"]),
                                         ("karpenter.sh/capacity-type", "In", ["on-demand", "spot"]),
                                         (K + "instance-category", "In", ["c", "m", "r"]),
                                         (K + "instance-generation", "Gt", ["4"])])]
    kinds = [_type_named(catalog, f"{f}.{s}") for f in ("m5", "c5", "r5") for s in ("large", "xlarge", "2xlarge", "4xlarge")]
    existing, bound = [], []
    for e in range(n_existing):
        ti = kinds[int(rng.integers(0, len(kinds)))]
        it = catalog[ti]
        name = f"node-{e:05d}"
        labels = node_labels(it, e % 3, "on-demand", "default", name)
        alloc = it.allocatable()
        used = {"cpu": 0, "memory": 0, "pods": 0}
        deps = set()
        for _ in range(64):
            j = int(rng.integers(0, n_deployments))
            if j in deps:
                continue
            rq = shapes[j].requests
            if any(used[r] + rq[r] > prefill * alloc[r] for r in used):
                break
            deps.add(j)
            for r in used:
                used[r] += rq[r]
            bound.append((shapes[j].namespace, dict(shapes[j].labels), e))
        avail = {r: alloc[r] - used[r] for r in used}
        existing.append(ExistingNode(name, labels, avail, {}, [], True))
    return Problem([catalog], pools, shapes, pod_shape, creation, uid, existing=existing, bound_pods=bound,
                   name=f"config3-{n}")


def random_topology_problem(catalog, seed, n_types=80, n_pods=240, n_existing=12, n_shapes=10, n_pools=2,
                            multi_terms=0.0, pns=0.0):
    """Randomized topology-spread scenario: zone / hostname / capacity-type keys, maxSkew 1-3, minDomains,
    ScheduleAnyway (relaxed away), selectors on own / other deployments / nil / expressions, node affinity
    and taint inclusion policies, zone-restricted pools and pods, bound pods seeding the counts.
    multi_terms: the share of shapes with 2-3 required node-affinity terms, the first often unsatisfiable, so that
    relaxation removes terms and re-creates the shapes' spread groups (Topology.Update)."""
    rng = np.random.default_rng(seed)
    idx = np.sort(rng.choice(len(catalog), size=min(n_types, len(catalog)), replace=False))
    cat = [catalog[i] for i in idx]
    cat = [it for it in cat if any(o.available for o in it.offerings)]
    pools = []
    for i in range(n_pools):
        reqs = [("karpenter.sh/capacity-type", "In", ["on-demand", "spot"] if rng.random() < 0.7 else ["spot"])]
        if rng.random() < 0.4:
            reqs.append((ZONE_KEY, "In", list(rng.choice(ZONES, size=2, replace=False))))
        taints = [("dedicated", f"team{i}", "NoSchedule")] if rng.random() < 0.3 else []
        limits = {"cpu": int(rng.integers(20, 400)) * 1000} if rng.random() < 0.3 else {}
        pools.append(NodePool(f"pool-{i}", int(rng.integers(0, 4)), 0, reqs, taints=taints, limits=limits))
    apps = [f"app-{j}" for j in range(n_shapes)]
    shapes = []
    for j in range(n_shapes):
        sh = PodShape(req_res(int(rng.choice([100, 250, 500, 1000, 2000])), int(rng.choice([128, 512, 1024, 2048]))),
                      labels={"app": apps[j], "tier": str(rng.choice(["web", "db"]))}, namespace=str(rng.choice(["a", "b"])))
        if rng.random() < 0.2:
            sh.node_selector = {ZONE_KEY: str(rng.choice(ZONES))}
        if rng.random() < 0.2:
            sh.required_terms = [[("karpenter.sh/capacity-type", "In", [str(rng.choice(["spot", "on-demand"]))])]]
        if multi_terms and rng.random() < multi_terms:
            pool_terms = [[(K + "instance-category", "In", ["x"])],  # x1 / x2 only: often unsatisfiable, relaxed away
                          [("karpenter.sh/capacity-type", "In", [str(rng.choice(["spot", "on-demand"]))])],
                          [(ZONE_KEY, "In", [str(rng.choice(ZONES))])],
                          [(K + "instance-category", "In", ["c", "m"])],
                          [(ZONE_KEY, "NotIn", [str(rng.choice(ZONES))]), (K + "instance-generation", "Gt", ["3"])]]
            pick = rng.choice(len(pool_terms), size=int(rng.integers(2, 4)), replace=False)
            if rng.random() < 0.6 and 0 not in pick:
                pick[0] = 0
            sh.required_terms = [pool_terms[int(i)] for i in pick]
        if rng.random() < 0.2:
            sh.preferred_terms = [(int(rng.integers(1, 100)), [(ZONE_KEY, "In", [str(rng.choice(ZONES))])])]
        if rng.random() < 0.3:
            sh.tolerations = [("dedicated", "Exists", "", "NoSchedule")]
        for _ in range(int(rng.integers(1, 3))):
            r = rng.random()
            if r < 0.6:
                sel = LabelSelector(match_labels={"app": apps[j]})
            elif r < 0.75:
                sel = LabelSelector(match_labels={"app": apps[int(rng.integers(0, n_shapes))]})
            elif r < 0.85:
                sel = LabelSelector(match_expressions=[("tier", "In", ["web"]), ("app", "NotIn", [apps[0]])])
            elif r < 0.93:
                sel = LabelSelector(match_expressions=[("app", "Exists", [])])
            else:
                sel = None
            key = str(rng.choice([ZONE_KEY, ZONE_KEY, HOST_KEY, HOST_KEY, "karpenter.sh/capacity-type"]))
            sh.topology_spread.append(TopologySpread(
                key, int(rng.choice([1, 1, 2, 3])), sel,
                "ScheduleAnyway" if rng.random() < 0.25 else "DoNotSchedule",
                int(rng.choice([2, 3, 4])) if rng.random() < 0.15 else None,
                "Ignore" if rng.random() < 0.15 else None,
                "Honor" if rng.random() < 0.2 else None))
        shapes.append(sh)
    existing, bound = [], []
    for e in range(n_existing):
        it = cat[int(rng.integers(0, len(cat)))]
        name = f"node-{e:05d}"
        labels = node_labels(it, int(rng.integers(0, 3)), str(rng.choice(["spot", "on-demand"])),
                             pools[int(rng.integers(0, n_pools))].name, name)
        alloc = it.allocatable()
        frac = float(rng.uniform(0.2, 0.9))
        avail = {k: int(v * frac) for k, v in alloc.items() if k in ("cpu", "memory", "pods")}
        existing.append(ExistingNode(name, labels, avail, {},
                                     [("dedicated", "team0", "NoSchedule")] if rng.random() < 0.15 else [],
                                     bool(rng.random() < 0.9)))
        for _ in range(int(rng.integers(0, 4))):
            j = int(rng.integers(0, n_shapes))
            bound.append((shapes[j].namespace, dict(shapes[j].labels), e))
    s, c, u = _pods(rng, n_pods, len(shapes))
    if pns:
        add_prefer_no_schedule(seed, pools, shapes, existing, pns)
    return Problem([cat], pools, shapes, s, c, u, existing=existing, bound_pods=bound, name=f"random-topology-{seed}")


def add_prefer_no_schedule(seed, pools, shapes, nodes, share):
    """Sprinkle PreferNoSchedule taints over a generated problem (its own rng, so the base scenario is unchanged):
    a share of the NodePools and existing nodes get a `soft=<name>:PreferNoSchedule` taint (upstream NewScheduler
    then turns on Preferences.ToleratePreferNoSchedule: pods relax to tolerate them last), and some shapes carry the
    exact toleration the relaxation would add (no extra level) or a key-specific one."""
    rng = np.random.default_rng(seed + 7919)
    for i, p in enumerate(pools):
        if rng.random() < share:
            p.taints = list(p.taints or []) + [("soft", f"p{i}", "PreferNoSchedule")]
    for n in nodes:
        if rng.random() < share:
            n.taints = list(n.taints or []) + [("soft", "node", "PreferNoSchedule")]
    for sh in shapes:
        u = rng.random()
        if u < 0.1:
            sh.tolerations = list(sh.tolerations or []) + [("", "Exists", "", "PreferNoSchedule")]
        elif u < 0.2:
            sh.tolerations = list(sh.tolerations or []) + [("soft", "Exists", "", "PreferNoSchedule")]


# ------------------------------------------------------------------------------------------------
# randomized parity scenarios (oracle vs device), small enough for the set-based oracle
# ------------------------------------------------------------------------------------------------
def random_problem(catalog, seed, n_types=120, n_pods=300, n_pools=3, n_existing=0, n_shapes=24, n_catalogs=1,
                   pns=0.0):
    """Random scenario. n_catalogs > 1: pool i resolves GetInstanceTypes to catalogue i % n_catalogs, each a
    different random subset of the docs catalogue (multi-NodeClass clusters). pns: the share of pools and existing
    nodes with a PreferNoSchedule taint (add_prefer_no_schedule)."""
    rng = np.random.default_rng(seed)
    idx = np.sort(rng.choice(len(catalog), size=min(n_types, len(catalog)), replace=False))
    cat = [catalog[i] for i in idx]
    cats = [cat]
    for _ in range(1, n_catalogs):
        ix = np.sort(rng.choice(len(catalog), size=min(n_types, len(catalog)), replace=False))
        cats.append([catalog[i] for i in ix])
    fams = sorted({r[2][0] for it in cat for r in it.requirements if r[0] == K + "instance-family" and r[2]})

    def rand_req(for_pool):
        kind = rng.integers(0, 14)
        if kind == 0:
            return (K + "instance-category", "In", list(rng.choice(["c", "m", "r", "t", "g", "x"], size=2, replace=False)))
        if kind == 1:
            return (K + "instance-category", "NotIn", [str(rng.choice(["c", "m", "r", "t"]))])
        if kind == 2:
            return (K + "instance-cpu", "Gt", [str(int(rng.choice([1, 2, 3, 4, 8, 16])))])
        if kind == 3:
            return (K + "instance-cpu", "Lt", [str(int(rng.choice([4, 8, 16, 33, 64])))])
        if kind == 4:
            return ("kubernetes.io/arch", "In", [str(rng.choice(["amd64", "arm64"]))])
        if kind == 5:
            return ("kubernetes.io/arch", "NotIn", ["arm64"])
        if kind == 6:
            return ("topology.kubernetes.io/zone", "In", list(rng.choice(ZONES, size=int(rng.integers(1, 3)), replace=False)))
        if kind == 7:
            return ("topology.kubernetes.io/zone", "NotIn", [str(rng.choice(ZONES))])
        if kind == 8:
            return ("karpenter.sh/capacity-type", "In", list(rng.choice(["spot", "on-demand"], size=int(rng.integers(1, 3)), replace=False)))
        if kind == 9:
            return (K + "instance-gpu-manufacturer", "DoesNotExist", [])
        if kind == 10:
            return (K + "instance-local-nvme", "Exists", [])
        if kind == 11:
            return (K + "instance-generation", "Gt", [str(int(rng.integers(1, 6)))])
        if kind == 12 and fams:
            return (K + "instance-family", "In" if rng.random() < 0.5 else "NotIn",
                    list(rng.choice(fams, size=min(len(fams), int(rng.integers(1, 6))), replace=False)))
        return (K + "instance-hypervisor", "In", ["nitro"])

    pools = []
    for i in range(n_pools):
        reqs = [rand_req(True) for _ in range(int(rng.integers(0, 3)))]
        if rng.random() < 0.15:
            reqs.append((K + "instance-family", "Exists", [], int(rng.integers(2, 5))))  # minValues
        taints = [("dedicated", f"team{i}", "NoSchedule")] if rng.random() < 0.3 else []
        limits = {"cpu": int(rng.integers(8, 200)) * 1000} if rng.random() < 0.5 else {}
        daemon = {"cpu": int(rng.choice([0, 100, 250])), "memory": 64 * MI * 1000, "pods": 1000} if rng.random() < 0.5 else {}
        pools.append(NodePool(f"pool-{i}", int(rng.integers(0, 4)), i % n_catalogs, reqs, labels={"team": f"t{i % 2}"},
                              taints=taints, limits=limits, daemon_requests=daemon))
    shapes = []
    for s in range(n_shapes):
        sh = PodShape(req_res(int(rng.choice(CPU_GRID)), int(rng.choice(MEM_GRID))))
        r = rng.random()
        if r < 0.2:
            sh.node_selector = {"topology.kubernetes.io/zone": str(rng.choice(ZONES))}
        elif r < 0.3:
            sh.node_selector = {"team": f"t{int(rng.integers(0, 3))}"}
        if rng.random() < 0.4:
            sh.required_terms = [[rand_req(False) for _ in range(int(rng.integers(1, 3)))]
                                 for _ in range(int(rng.integers(1, 3)))]
        if rng.random() < 0.25:
            sh.preferred_terms = [(int(rng.integers(1, 100)), [rand_req(False)]) for _ in range(int(rng.integers(1, 3)))]
        if rng.random() < 0.3:
            sh.tolerations = [("dedicated", "Exists", "", "NoSchedule")] if rng.random() < 0.5 else \
                [("dedicated", "Equal", f"team{int(rng.integers(0, n_pools))}", "")]
        if rng.random() < 0.05:
            sh.requests["nvidia.com/gpu"] = 1000
        shapes.append(sh)
    existing = []
    for e in range(n_existing):
        it = cat[int(rng.integers(0, len(cat)))]
        labels = {r[0]: r[2][0] for r in it.requirements if r[1] == "In" and len(r[2]) == 1}
        labels["topology.kubernetes.io/zone"] = str(rng.choice(ZONES))
        labels["karpenter.sh/capacity-type"] = str(rng.choice(["spot", "on-demand"]))
        labels["karpenter.sh/nodepool"] = pools[int(rng.integers(0, n_pools))].name
        labels["kubernetes.io/hostname"] = f"node-{e:05d}"
        alloc = it.allocatable()
        frac = float(rng.uniform(0.1, 0.9))
        avail = {k: int(v * frac) for k, v in alloc.items() if k in ("cpu", "memory", "pods")}
        existing.append(ExistingNode(f"node-{e:05d}", labels, avail, {},
                                     [("dedicated", "team0", "NoSchedule")] if rng.random() < 0.1 else [],
                                     bool(rng.random() < 0.9)))
    s, c, u = _pods(rng, n_pods, len(shapes))
    if pns:
        add_prefer_no_schedule(seed, pools, shapes, existing, pns)
    return Problem(cats, pools, shapes, s, c, u, existing=existing, name=f"random-{seed}")


# ------------------------------------------------------------------------------------------------
# config 4: a running cluster for multi-node consolidation (10k nodes, 8-40 pods per node)
# ------------------------------------------------------------------------------------------------
C4_CPU = [250, 500, 1000, 2000]
C4_MEM = [256, 512, 1024, 2048, 4096]


def node_labels(it, zone_i, capacity_type, nodepool, hostname):
    """Labels a launched node carries: the type's single-valued requirements + offering + NodePool."""
    labels = {r[0]: r[2][0] for r in it.requirements if r[1] == "In" and len(r[2]) == 1}
    labels["topology.kubernetes.io/zone"] = ZONES[zone_i]
    labels["topology.k8s.aws/zone-id"] = ZONE_IDS[zone_i]
    labels["karpenter.sh/capacity-type"] = capacity_type
    labels["karpenter.sh/nodepool"] = nodepool
    labels["kubernetes.io/hostname"] = hostname
    return labels


def config4(catalog, n_nodes=10_000, seed=4, n_shapes=32, pods_min=8, pods_max=40, fill=(0.97, 1.0), topup=True,
            loose=0.004, loose_fill=(0.4, 0.8)):
    """A cluster of n_nodes c/m/r nodes (2-16 vCPU, 3 AZ, 80% on-demand) running 8-40 pods each: a random start,
    then topped up with the largest shapes that fit, to 97-100% of the binding resource (0.4% of the nodes stay
    40-80% used: the cluster's usable slack), so that the displaced pods of a candidate subset often exceed the remaining
    slack: the sweep then sees delete, replace and no-op decisions (at 70-98% fill every subset was a delete);
    2 NodePools without limits. Candidates are sorted by disruption cost (fewer pods first, then name:
    R:website/content/en/preview/concepts/disruption.md:101-103)."""
    rng = np.random.default_rng(seed)
    pools = [
        NodePool("default", 10, 0, [("karpenter.sh/capacity-type", "In", ["on-demand", "spot"]),
                                    (K + "instance-category", "In", ["c", "m", "r"]),
                                    (K + "instance-generation", "Gt", ["4"])]),
        NodePool("burst", 1, 0, [("karpenter.sh/capacity-type", "In", ["spot"]),
                                 (K + "instance-category", "In", ["c", "m"])]),
    ]

    def req_val(it, key):
        for r in it.requirements:
            if r[0] == key and r[1] == "In" and len(r[2]) == 1:
                return r[2][0]
        return None

    pool_types = []
    for i, it in enumerate(catalog):
        cat_ = req_val(it, K + "instance-category")
        gen = req_val(it, K + "instance-generation")
        cpu_n = int(req_val(it, K + "instance-cpu") or 0)
        if cat_ in ("c", "m", "r") and gen and int(gen) > 4 and 2 <= cpu_n <= 16 \
                and req_val(it, "kubernetes.io/arch") == "amd64" and any(o.available for o in it.offerings):
            pool_types.append(i)
    shapes = []
    for i in range(n_shapes):
        sh = PodShape(req_res(int(rng.choice(C4_CPU)), int(rng.choice(C4_MEM))))
        if i % 8 == 7:
            sh.node_selector = {"topology.kubernetes.io/zone": ZONES[(i // 8) % 3]}
        elif i % 8 == 6:
            sh.required_terms = [[("kubernetes.io/arch", "In", ["amd64"])]]
        shapes.append(sh)
    shape_zone = [ZONES.index(sh.node_selector["topology.kubernetes.io/zone"]) if sh.node_selector else -1
                  for sh in shapes]
    topup_order = sorted(range(n_shapes), key=lambda i: (-shapes[i].requests["cpu"], -shapes[i].requests["memory"], i))
    nodes = []
    pod_shape, pod_creation, pod_uid = [], [], []
    for n in range(n_nodes):
        it = catalog[int(rng.choice(pool_types))]
        zone_i = int(rng.integers(0, 3))
        ct = "spot" if rng.random() < 0.2 else "on-demand"
        name = f"node-{n:06d}"
        labels = node_labels(it, zone_i, ct, "default", name)
        alloc = it.allocatable()
        is_loose = rng.random() < loose  # an underutilised node (no top-up): the cluster's usable slack
        frac = float(rng.uniform(*(loose_fill if is_loose else fill)))
        k = int(rng.integers(pods_min, pods_max + 1))
        used = {"cpu": 0, "memory": 0, "pods": 0}
        pods = []
        for _ in range(4 * k):
            if len(pods) >= k:
                break
            s_i = int(rng.integers(0, n_shapes))
            if shape_zone[s_i] not in (-1, zone_i):
                continue
            rq = shapes[s_i].requests
            if any(used[r] + rq[r] > frac * alloc[r] for r in used):
                continue
            for r in used:
                used[r] += rq[r]
            pods.append(len(pod_shape))
            pod_shape.append(s_i)
            pod_creation.append(1_750_000_000 + int(rng.integers(0, 86_400)))
            pod_uid.append(int(rng.integers(0, np.iinfo(np.int64).max)))
        if topup and not is_loose:  # pack the rest: the largest shapes that still fit under frac, up to pods_max pods
            for s_i in topup_order:
                if shape_zone[s_i] not in (-1, zone_i):
                    continue
                rq = shapes[s_i].requests
                while len(pods) < pods_max and not any(used[r] + rq[r] > frac * alloc[r] for r in used):
                    for r in used:
                        used[r] += rq[r]
                    pods.append(len(pod_shape))
                    pod_shape.append(s_i)
                    pod_creation.append(1_750_000_000 + int(rng.integers(0, 86_400)))
                    pod_uid.append(int(rng.integers(0, np.iinfo(np.int64).max)))
        avail = {r: alloc[r] - used[r] for r in used}
        nodes.append(ClusterNode(ExistingNode(name, labels, avail, {}, [], True), 0, catalog.index(it), pods))
    cands = sorted(range(n_nodes), key=lambda i: (len(nodes[i].pods), nodes[i].node.name))
    return Cluster([catalog], pools, nodes, shapes, np.asarray(pod_shape, dtype=np.uint32),
                   np.asarray(pod_creation, dtype=np.int64), np.asarray(pod_uid, dtype=np.uint64),
                   candidates=cands, name=f"config4-{n_nodes}")


def consolidation_subsets(cluster, n_random, seed=44, max_size=100, prefixes=True):
    """MultiNodeConsolidation probes: every prefix candidates[0:k] (k = 2..100) and n_random random
    subsets of 2..max_size candidates (each kept in candidate order)."""
    rng = np.random.default_rng(seed)
    c = cluster.candidates
    out = [c[:k] for k in range(2, min(len(c), max_size) + 1)] if prefixes else []
    pos = {n: i for i, n in enumerate(c)}
    for _ in range(n_random):
        k = int(rng.integers(2, min(len(c), max_size) + 1))
        pick = rng.choice(len(c), size=k, replace=False)
        out.append([c[i] for i in sorted(pick)])
    del pos
    return out


def spread_cluster(catalog, n_nodes, seed=4):
    """Config 4 with topology spread: every shape labelled app-(i % 8), every other shape zone-spread (maxSkew 1,
    DoNotSchedule) over its app. The batched sim kernels do not model spread, so kp_cluster_prepare takes the general
    path (each subset's SimulateScheduling a Solve on the device, the remaining nodes' pods counted)."""
    cl = config4(catalog, n_nodes=n_nodes, seed=seed)
    for i, sh in enumerate(cl.shapes):
        sh.labels = dict(sh.labels or {}, app=f"app-{i % 8}")
        if i % 2 == 0:
            sh.topology_spread = [TopologySpread("topology.kubernetes.io/zone", 1, LabelSelector({"app": f"app-{i % 8}"}),
                                                 "DoNotSchedule")]
    return cl


def random_cluster(catalog, seed, n_nodes=60, n_types=80, n_shapes=16, n_pools=2, pns=0.0):
    """Randomized consolidation scenario: pools with taints / daemonsets / minValues, pods with selectors,
    NotIn / Gt affinities and relaxable preferences on keys every node carries, spot and uninitialized
    nodes."""
    rng = np.random.default_rng(seed)
    idx = np.sort(rng.choice(len(catalog), size=min(n_types, len(catalog)), replace=False))
    cat = [catalog[i] for i in idx]
    cat = [it for it in cat if any(o.available for o in it.offerings)
           and any(r[0] == K + "instance-category" for r in it.requirements)]

    def rand_req():
        kind = rng.integers(0, 8)
        if kind == 0:
            return (K + "instance-category", "In", list(rng.choice(["c", "m", "r", "t"], size=2, replace=False)))
        if kind == 1:
            return (K + "instance-category", "NotIn", [str(rng.choice(["c", "m", "r", "t"]))])
        if kind == 2:
            return ("kubernetes.io/arch", "In", [str(rng.choice(["amd64", "arm64"]))])
        if kind == 3:
            return ("topology.kubernetes.io/zone", "NotIn", [str(rng.choice(ZONES))])
        if kind == 4:
            return ("karpenter.sh/capacity-type", "In", list(rng.choice(["spot", "on-demand"], size=int(rng.integers(1, 3)), replace=False)))
        if kind == 5:
            return (K + "instance-cpu", "Gt", [str(int(rng.choice([1, 2, 4])))])
        if kind == 6:
            return ("topology.kubernetes.io/zone", "In", list(rng.choice(ZONES, size=2, replace=False)))
        return ("kubernetes.io/arch", "NotIn", ["arm64"])

    pools = []
    for i in range(n_pools):
        reqs = [rand_req() for _ in range(int(rng.integers(0, 3)))]
        if rng.random() < 0.2:
            reqs.append((K + "instance-family", "Exists", [], int(rng.integers(2, 4))))
        taints = [("dedicated", f"team{i}", "NoSchedule")] if rng.random() < 0.3 else []
        daemon = {"cpu": int(rng.choice([0, 100, 250])), "memory": 64 * MI * 1000, "pods": 1000} if rng.random() < 0.5 else {}
        pools.append(NodePool(f"pool-{i}", int(rng.integers(0, 4)), 0, reqs, taints=taints, daemon_requests=daemon))
    shapes = []
    for s in range(n_shapes):
        sh = PodShape(req_res(int(rng.choice([50, 100, 250, 500, 1000])), int(rng.choice([64, 256, 512, 1024, 2048]))))
        r = rng.random()
        if r < 0.2:
            sh.node_selector = {"topology.kubernetes.io/zone": str(rng.choice(ZONES))}
        if rng.random() < 0.3:
            sh.required_terms = [[rand_req()] for _ in range(int(rng.integers(1, 3)))]
        if rng.random() < 0.2:
            sh.preferred_terms = [(int(rng.integers(1, 100)), [rand_req()])]
        if rng.random() < 0.3:
            sh.tolerations = [("dedicated", "Exists", "", "NoSchedule")]
        shapes.append(sh)
    nodes, pod_shape, pod_creation, pod_uid = [], [], [], []
    for n in range(n_nodes):
        ti = int(rng.integers(0, len(cat)))
        it = cat[ti]
        zone_i = int(rng.integers(0, 3))
        pool = pools[int(rng.integers(0, n_pools))]
        name = f"node-{n:05d}"
        labels = node_labels(it, zone_i, "spot" if rng.random() < 0.3 else "on-demand", pool.name, name)
        alloc = it.allocatable()
        frac = float(rng.uniform(0.3, 0.95))
        used = {"cpu": 0, "memory": 0, "pods": 0}
        pods = []
        for _ in range(int(rng.integers(0, 30))):
            s_i = int(rng.integers(0, n_shapes))
            rq = shapes[s_i].requests
            if any(used[r] + rq[r] > frac * alloc[r] for r in used):
                continue
            for r in used:
                used[r] += rq[r]
            pods.append(len(pod_shape))
            pod_shape.append(s_i)
            pod_creation.append(1_750_000_000 + int(rng.integers(0, 600)))
            pod_uid.append(int(rng.integers(0, np.iinfo(np.int64).max)))
        avail = {r: alloc[r] - used[r] for r in used}
        nodes.append(ClusterNode(ExistingNode(name, labels, avail, {}, list(pool.taints), bool(rng.random() < 0.95)),
                                 0, ti, pods))
    cands = sorted(range(n_nodes), key=lambda i: (len(nodes[i].pods), nodes[i].node.name))
    if pns:  # (nodes keep their pool's taints; a PreferNoSchedule pool's nodes carry its taint too)
        add_prefer_no_schedule(seed, pools, shapes, [], pns)
        for n in nodes:
            pool = next(p for p in pools if p.name == n.node.labels["karpenter.sh/nodepool"])
            n.node.taints = list(pool.taints)
    return Cluster([cat], pools, nodes, shapes, np.asarray(pod_shape, dtype=np.uint32),
                   np.asarray(pod_creation, dtype=np.int64), np.asarray(pod_uid, dtype=np.uint64),
                   candidates=cands, name=f"random-cluster-{seed}")


# ------------------------------------------------------------------------------------------------
# launch-side selection (instance.DefaultProvider.Create) requests
# ------------------------------------------------------------------------------------------------
def single_pod_problem(catalog, pool_reqs, requests, name="single-pod"):
    """One pending pod on one NodePool (the reference's launch tests: R:pkg/providers/instancetype/suite_test.go)."""
    rng = np.random.default_rng(0)
    s, c, u = _pods(rng, 1, 1)
    return Problem([catalog], [NodePool("default", 0, 0, list(pool_reqs))], [PodShape(dict(requests))], s, c, u,
                   name=name)


def random_launch_requests(catalog, n, seed):
    """n random launch requests: NodeClaim-like requirements (capacity type, zones, categories, cpu bounds, arch,
    minValues, GPU manufacturer), requests and instance-type lists (random subsets, the whole catalogue, empty)."""
    rng = np.random.default_rng(seed)
    T = len(catalog)
    fams = sorted({r[2][0] for it in catalog for r in it.requirements if r[0] == K + "instance-family" and r[2]})
    out = []
    for _ in range(n):
        reqs = []
        k = rng.random()
        if k < 0.25:
            reqs.append(("karpenter.sh/capacity-type", "In", ["spot", "on-demand"]))
        elif k < 0.45:
            reqs.append(("karpenter.sh/capacity-type", "In", ["on-demand"]))
        elif k < 0.6:
            reqs.append(("karpenter.sh/capacity-type", "In", ["spot"]))
        elif k < 0.65:
            reqs.append(("karpenter.sh/capacity-type", "NotIn", ["spot"]))
        if rng.random() < 0.3:
            reqs.append(("topology.kubernetes.io/zone", "In", list(rng.choice(ZONES, size=int(rng.integers(1, 3)), replace=False))))
        elif rng.random() < 0.1:
            reqs.append(("topology.kubernetes.io/zone", "NotIn", [str(rng.choice(ZONES))]))
        if rng.random() < 0.3:
            reqs.append((K + "instance-category", "In", list(rng.choice(["c", "m", "r", "g", "p", "t", "x", "i"],
                                                                       size=int(rng.integers(1, 4)), replace=False))))
        if rng.random() < 0.2:
            reqs.append((K + "instance-cpu", "Gt", [str(int(rng.choice([1, 3, 7, 15])))]))
        if rng.random() < 0.15:
            reqs.append((K + "instance-cpu", "Lt", [str(int(rng.choice([8, 17, 33, 97])))]))
        if rng.random() < 0.3:
            reqs.append(("kubernetes.io/arch", "In", [str(rng.choice(["amd64", "arm64"]))]))
        if rng.random() < 0.1:
            reqs.append((K + "instance-gpu-manufacturer", "In", ["nvidia"]))
        if rng.random() < 0.1 and fams:
            reqs.append((K + "instance-family", "In" if rng.random() < 0.7 else "NotIn",
                         list(rng.choice(fams, size=min(len(fams), int(rng.integers(2, 12))), replace=False)),
                         int(rng.integers(1, 5)) if rng.random() < 0.7 else None))
        if rng.random() < 0.05:
            reqs.append((K + "instance-size", "Exists", [], 2))
        res = req_res(int(rng.choice(CPU_GRID + [8000, 16000])), int(rng.choice(MEM_GRID + [32768])))
        if any(r[0] == K + "instance-gpu-manufacturer" for r in reqs) and rng.random() < 0.5:
            res["nvidia.com/gpu"] = 1000
        u = rng.random()
        if u < 0.05:
            lst = []
        elif u < 0.15:
            lst = list(range(T))
        else:
            lst = sorted(rng.choice(T, size=int(rng.integers(1, min(T, 300))), replace=False).tolist())
            if rng.random() < 0.5:
                rng.shuffle(lst)
        out.append((reqs, res, [int(t) for t in lst]))
    return out


# ------------------------------------------------------------------------------------------------
# feasibility rows: distinct (requirements, requests) queries (SURVEY §8d unit = one (pod shape, type) pair)
# ------------------------------------------------------------------------------------------------
def distinct_queries(catalog, n, seed=8):
    """n pairwise-distinct CompatibleAvailableFilter rows, the requirement mixes of deployments in a large cluster:
    zone / capacity-type / category / arch / cpu bounds / GPU / family constraints and cpu-memory(-GPU) requests.
    Distinctness is exact (a row repeats no other row's requirements + requests)."""
    rng = np.random.default_rng(seed)
    fams = sorted({r[2][0] for it in catalog for r in it.requirements if r[0] == K + "instance-family" and r[2]})
    cats = ["c", "m", "r", "t", "g", "p", "x", "i", "z", "d"]
    seen, out = set(), []
    while len(out) < n:
        reqs = []
        if rng.random() < 0.35:
            reqs.append(("topology.kubernetes.io/zone", "In", sorted(rng.choice(ZONES, size=int(rng.integers(1, 3)), replace=False).tolist())))
        if rng.random() < 0.5:
            reqs.append(("karpenter.sh/capacity-type", "In", sorted(rng.choice(["spot", "on-demand"], size=int(rng.integers(1, 3)), replace=False).tolist())))
        if rng.random() < 0.5:
            reqs.append((K + "instance-category", "In" if rng.random() < 0.8 else "NotIn",
                         sorted(rng.choice(cats, size=int(rng.integers(1, 4)), replace=False).tolist())))
        if rng.random() < 0.3:
            reqs.append(("kubernetes.io/arch", "In", [str(rng.choice(["amd64", "arm64"]))]))
        if rng.random() < 0.3:
            reqs.append((K + "instance-cpu", "Gt", [str(int(rng.choice([1, 3, 7, 15, 31])))]))
        if rng.random() < 0.2:
            reqs.append((K + "instance-cpu", "Lt", [str(int(rng.choice([8, 17, 33, 65, 97])))]))
        if rng.random() < 0.15:
            reqs.append((K + "instance-generation", "Gt", [str(int(rng.integers(2, 7)))]))
        if rng.random() < 0.1 and fams:
            reqs.append((K + "instance-family", "In", sorted(rng.choice(fams, size=int(rng.integers(2, 16)), replace=False).tolist())))
        if rng.random() < 0.1:
            reqs.append((K + "instance-gpu-manufacturer", "DoesNotExist", []))
        res = req_res(int(rng.integers(1, 400)) * 50, int(rng.integers(1, 512)) * 64)
        if rng.random() < 0.05:
            res["nvidia.com/gpu"] = 1000 * int(rng.choice([1, 2, 4]))
        key = (tuple((k, op, tuple(v)) for k, op, v in reqs), tuple(sorted(res.items())))
        if key in seen:
            continue
        seen.add(key)
        out.append((reqs, res))
    return out


def with_disruption_state(cluster, seed, n_deleting=3, n_pending=6, cpu_limit_m=None):
    """A copy of a consolidation cluster with the rest of SimulateScheduling's inputs: n_deleting nodes marked for
    deletion (dropped from the candidates; their pods join every simulation), n_pending provisionable pods bound to
    no node (shapes of the cluster, a quarter of them oversized so they cannot schedule), and optionally a remaining
    cpu limit on every NodePool (kp_nodepool limits are remaining limits)."""
    import copy
    rng = np.random.default_rng(seed)
    cl = copy.deepcopy(cluster)
    order = rng.permutation(len(cl.nodes))[:n_deleting]
    for i in order:
        cl.nodes[int(i)].deleting = True
    dele = {int(i) for i in order}
    cl.candidates = [c for c in cl.candidates if c not in dele]
    n0 = len(cl.pod_shape)
    shapes = list(cl.shapes)
    new_shape = []
    for j in range(n_pending):
        if j % 4 == 3:  # fits no node and no instance type: a pending pod whose error must not block the decision
            shapes.append(PodShape(req_res(10_000_000, 64)))
            new_shape.append(len(shapes) - 1)
        else:
            new_shape.append(int(rng.integers(0, len(cluster.shapes))))
    cl.shapes = shapes
    cl.pod_shape = np.concatenate([cl.pod_shape, np.asarray(new_shape, dtype=cl.pod_shape.dtype)])
    cl.pod_creation = np.concatenate([cl.pod_creation, (1_750_000_000 + rng.integers(0, 600, size=n_pending)).astype(np.int64)])
    cl.pod_uid = np.concatenate([cl.pod_uid, rng.integers(0, np.iinfo(np.int64).max, size=n_pending, dtype=np.int64).astype(np.uint64)])
    cl.pending = list(range(n0, n0 + n_pending))
    if cpu_limit_m is not None:
        for np_ in cl.nodepools:
            np_.limits = {"cpu": int(cpu_limit_m)}
    cl.name = f"{cluster.name}+disruption-state"
    return cl
