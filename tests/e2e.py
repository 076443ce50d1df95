"""The reference's e2e suites (test/suites/scheduling, test/suites/consolidation), restated as a cluster simulation over
either backend — TEST INFRASTRUCTURE.

The e2e tests run Karpenter against EC2: provision Deployments, scale them, let the disruption controller consolidate,
and assert on the nodes that remain. This module keeps the same loop with every AWS and kube-scheduler step replaced by
a small deterministic model, and the Karpenter steps computed by the backend under test:

  backend "device"  Solve (kp_solve), launch selection (kp_launch_prepare/run), consolidation decisions
                    (kp_cluster_prepare + kp_cluster_simulate through kpamd.disruption.Controller) on the GPU
  backend "oracle"  the same three on the CPU restatement (oracle/liboracle.so)

The model (what the e2e environment does outside Karpenter):
  catalogue        the 919-type docs catalogue (kpamd.catalog.build_catalog: test-zone-1a..c, splitmix64 spot prices),
                   the EC2NodeClass's capacity reservations with their available counts (instances launched into a
                   reservation use it up: the catalogue is rebuilt with the remaining counts)
  CreateFleet      the request's overrides (kp_launch's capacity type and (type, zone) list); the instance is the
                   cheapest override (lowest-price allocation; ties: the first), a reserved launch needs room left in
                   the reservation; every launch succeeds (no ICE here: tests/scenarios.py covers ICE)
  kube-scheduler   a pod binds where Karpenter's Solve placed it: an existing node, or the NodeClaim's new node
  ReplicaSet       scale-down deletes the pods on the nodes holding most replicas first, newest first (the
                   controller's ActivePodsWithRanks order for ready pods with equal deletion cost)
  daemonsets       none (GetDaemonSetOverhead = 0: the e2e "1800m - daemonset overhead" pods are 1800m)
  consolidation    consolidateAfter 0 and no disruption budget; a command's candidates are replaced at once; the pods
                   of a DELETE / REPLACE go where the command's SimulateScheduling placed them (the Solve of the pending
                   pods plus the candidates' pods onto the other nodes, strict reservations), the replacement is
                   launched from its NodeClaim after filterByPrice (and filterOutSameType for a multi-node command;
                   spot-to-spot: spot offerings only, at least 15 options and the cheapest 15 kept), the feature gate
                   SpotToSpotConsolidation on as in the suites' install (R:test/hack/e2e_scripts/install_karpenter.sh:19)
"""
import collections
import math

import numpy as np

K = "karpenter.k8s.aws/"
ZONE = "topology.kubernetes.io/zone"
ZONE_ID = "topology.k8s.aws/zone-id"
CT = "karpenter.sh/capacity-type"
IT = "node.kubernetes.io/instance-type"
HOST = "kubernetes.io/hostname"
RID = K + "capacity-reservation-id"
RTYPE = K + "capacity-reservation-type"
POOL = "karpenter.sh/nodepool"
NOT_BURSTABLE = (K + "instance-family", "NotIn", ["t2", "t3", "c1", "t3a", "t4g", "a1"])


def default_nodepool(name="default"):
    """env.DefaultNodePool (R:test/pkg/environment/common/environment.go:133-175): linux, on-demand, categories c/m/r,
    generation > 2, no a1."""
    from kpamd.model import NodePool
    return NodePool(name, 0, 0, [("kubernetes.io/os", "In", ["linux"]), (CT, "In", ["on-demand"]),
                                 (K + "instance-category", "In", ["c", "m", "r"]), (K + "instance-generation", "Gt", ["2"]),
                                 (K + "instance-family", "NotIn", ["a1"])])


def _offering_compatible(reqs, o):
    """Requirements.Compatible(offering requirements) on the offering keys (capacity type, zone, zone id, reservation
    id / type; an offering without a reservation is DoesNotExist on those keys)."""
    labels = {CT: o.capacity_type, ZONE: o.zone, ZONE_ID: o.zone_id, RID: o.reservation_id, RTYPE: o.reservation_type}
    for k, op, vals, *_ in reqs:
        if k not in labels:
            continue
        v = labels[k]
        if op == "In" and (v is None or v not in vals):
            return False
        if op == "NotIn" and v is not None and v in vals:
            return False
        if op == "Exists" and v is None:
            return False
        if op == "DoesNotExist" and v is not None:
            return False
    return True


def _has(reqs, key, value):
    """Requirements.Get(key).Has(value) (an absent key is Exists)."""
    for k, op, vals, *_ in reqs:
        if k != key:
            continue
        if (op == "In" and value not in vals) or (op == "NotIn" and value in vals) or op == "DoesNotExist":
            return False
    return True


def worst_launch_price(it, reqs, spot_only=False):
    """Offerings.Available().Compatible(reqs).WorstLaunchPrice: the most expensive offering of the first capacity type,
    in the order reserved, spot, on-demand, that has one (oracle/oracle.cpp WorstLaunchPrice)."""
    for ct in ("reserved", "spot", "on-demand"):
        if spot_only and ct != "spot":
            continue
        ps = [o.price for o in it.offerings if o.available and o.capacity_type == ct and _offering_compatible(reqs, o)]
        if ps:
            return max(ps)
    return math.inf


class OraclePlan:
    """The oracle behind ClusterPlan's simulate() (kpamd.disruption.Controller takes either)."""

    def __init__(self, cluster):
        self.cluster = cluster

    def simulate(self, subsets, multi_node=True):
        from oracle import pyoracle
        return pyoracle.simulate_batch(self.cluster, subsets, multi_node=multi_node)

    def close(self):
        pass


class Env:
    def __init__(self, backend, lib, ctx=None, reservations=(), spot_to_spot=True):
        from kpamd import catalog as cmod
        self.backend, self.lib, self.ctx = backend, lib, ctx
        self.cmod = cmod
        self.crs = collections.OrderedDict((cr.id, cr) for cr in reservations)
        self.pools = []
        self.shapes = []
        self.pod_shape, self.pod_created, self.pod_node, self.alive = [], [], [], []
        self.deployments = {}
        self.nodes = collections.OrderedDict()  # name -> {type, zone, ct, pool, rid, rtype}
        self.n_made = 0
        self.clock = 1_750_000_000
        self.spot_to_spot = spot_to_spot
        self._types, self._key, self._cat, self._seq = None, None, None, 0
        self.launches = []  # every CreateFleet: (node name, type name, zone, capacity type, NodeClaim requirements)
        self.commands = []  # every consolidation command applied

    # ---- the catalogue ---------------------------------------------------------------------------------------------
    def types(self):
        used = collections.Counter(n["rid"] for n in self.nodes.values() if n["rid"])
        crs = [self.cmod.CapacityReservation(c.id, c.instance_type, c.availability_zone, c.reservation_type,
                                             max(0, c.available_count - used[c.id])) for c in self.crs.values()]
        key = tuple((c.id, c.available_count) for c in crs)
        if self._types is None or key != self._key:
            self._types, self._key = self.cmod.build_catalog(self.lib, capacity_reservations=crs), key
            if self.backend == "device":
                import kpamd
                if self._cat is not None:
                    self._cat.close()
                self._seq += 1
                self._cat = kpamd.Catalog(self.ctx, self._types, seqnum=self._seq)
        return self._types

    def add_reservation(self, cr):
        """The EC2NodeClass selects one more capacity reservation (capacityReservationSelectorTerms)."""
        self.crs[cr.id] = cr

    def type_index(self, name):
        return next(i for i, t in enumerate(self.types()) if t.name == name)

    def close(self):
        if self._cat is not None:
            self._cat.close()
            self._cat = None

    # ---- workloads -------------------------------------------------------------------------------------------------
    def deploy(self, name, shape, replicas):
        self.shapes.append(shape)
        self.deployments[name] = (len(self.shapes) - 1, [])
        self.scale(name, replicas)

    def scale(self, name, replicas, seed=None):
        """Deployment.spec.replicas = replicas. seed: the pods to delete drawn at random instead (a scale-down spread
        over the nodes, which leaves them partly used rather than empty)."""
        s, pods = self.deployments[name]
        live = [p for p in pods if self.alive[p]]
        for _ in range(replicas - len(live)):  # new pods (pending)
            self.pod_shape.append(s)
            self.pod_created.append(self.clock)
            self.clock += 1
            self.pod_node.append(None)
            self.alive.append(True)
            pods.append(len(self.pod_shape) - 1)
        if replicas < len(live):  # ReplicaSet scale-down: most-doubled-up nodes first, then the newest pods
            rank = collections.Counter(self.pod_node[p] for p in live)
            order = sorted(live, key=lambda p: (self.pod_node[p] is not None, -rank[self.pod_node[p]],
                                                -self.pod_created[p]))
            if seed is not None:
                order = list(np.random.default_rng(seed).permutation(live))
            for p in order[:len(live) - replicas]:
                self.alive[p] = False
                self.pod_node[p] = None

    def pods_on(self, name):
        return [p for p in range(len(self.pod_shape)) if self.alive[p] and self.pod_node[p] == name]

    def pending(self):
        return [p for p in range(len(self.pod_shape)) if self.alive[p] and self.pod_node[p] is None]

    # ---- nodes -------------------------------------------------------------------------------------------------------
    def labels(self, name):
        n = self.nodes[name]
        it = self.types()[n["type"]]
        lab = {r[0]: r[2][0] for r in it.requirements if r[1] == "In" and len(r[2]) == 1}
        lab.update({ZONE: n["zone"], ZONE_ID: self.cmod.ZONE_IDS[self.cmod.ZONES.index(n["zone"])], CT: n["ct"],
                    POOL: self.pools[n["pool"]].name, HOST: name})
        lab.pop(RID, None)
        lab.pop(RTYPE, None)
        if n["rid"]:
            lab[RID], lab[RTYPE] = n["rid"], n["rtype"]
        return lab

    def allocatable(self, name):
        return self.types()[self.nodes[name]["type"]].allocatable()

    def _requested(self, pods):
        out = collections.Counter()
        for p in pods:
            out.update(self.shapes[self.pod_shape[p]].requests)
        return out

    def _existing(self, names):
        from kpamd.model import ExistingNode
        out, bound = [], []
        for e, name in enumerate(names):
            pods = self.pods_on(name)
            used = self._requested(pods)
            alloc = self.allocatable(name)
            out.append(ExistingNode(name, self.labels(name), {r: v - used.get(r, 0) for r, v in alloc.items()}, {},
                                    list(self.pools[self.nodes[name]["pool"]].taints), True))
            for p in pods:
                sh = self.shapes[self.pod_shape[p]]
                bound.append((sh.namespace, dict(sh.labels), e))
        return out, bound

    def _solve(self, pods, names):
        """Scheduler.Solve of `pods` onto the nodes `names` + new NodeClaims (the provisioner's scheduler: strict
        reservations). Returns the result dict."""
        from kpamd.model import Problem
        existing, bound = self._existing(names)
        prob = Problem([self.types()], self.pools, self.shapes, np.array([self.pod_shape[p] for p in pods], np.uint32),
                       np.array([self.pod_created[p] for p in pods], np.int64),
                       np.array([p + 1 for p in pods], np.uint64), existing=existing, bound_pods=bound,
                       name="e2e", reserved_offering_mode=1)
        if self.backend == "device":
            import kpamd
            self.types()
            return kpamd.Scheduler(self.ctx, prob, catalogs=[self._cat]).solve()
        from oracle import pyoracle
        return pyoracle.solve(prob)

    def _launch_select(self, reqs, requests, options):
        zones = list(self.cmod.ZONES)
        if self.backend == "device":
            import kpamd
            self.types()
            plan = kpamd.LaunchPlan(self.ctx, self._cat, [(reqs, requests, options)], zones)
            try:
                return plan.run(read=True)[0][0]
            finally:
                plan.close()
        from oracle import pyoracle
        return pyoracle.launch_select(self.types(), [(reqs, requests, options)], zones)[0]

    def _create(self, reqs, requests, options, pool):
        """CloudProvider.Create + the fake CreateFleet (module docstring). Returns the new node's name or None."""
        lr = self._launch_select(reqs, requests, options)
        if lr["status"] != 0:
            return None
        types = self.types()
        used = collections.Counter(n["rid"] for n in self.nodes.values() if n["rid"])
        best = None
        for t, z in lr["overrides"]:
            for o in types[t].offerings:
                if o.capacity_type != lr["capacity_type"] or o.zone != z or not o.available:
                    continue
                if o.reservation_id and self.crs[o.reservation_id].available_count - used[o.reservation_id] <= 0:
                    continue
                if best is None or o.price < best[0]:
                    best = (o.price, t, o)
        if best is None:
            return None
        _, t, o = best
        name = f"node-{self.n_made:04d}"
        self.n_made += 1
        self.nodes[name] = {"type": t, "zone": o.zone, "ct": o.capacity_type, "pool": pool,
                            "rid": o.reservation_id, "rtype": o.reservation_type}
        self.launches.append((name, types[t].name, o.zone, o.capacity_type, list(reqs)))
        return name

    def provision(self, rounds=4):
        """ExpectProvisioned until no pod is pending or a round makes no progress (a strict-reservation failure is
        retried on the next round, as the provisioner's next batch would)."""
        for _ in range(rounds):
            pods = self.pending()
            if not pods:
                return
            names = list(self.nodes)
            res = self._solve(pods, names)
            progress = False
            for i, pl in enumerate(res["placement"]):
                if pl <= -2:
                    self.pod_node[pods[i]] = names[-2 - int(pl)]
                    progress = True
            for nc in res["nodeclaims"]:
                name = self._create(nc["requirements"], nc["requests"], nc["options"], nc["nodepool"])
                if name is not None:
                    for i in nc["pods"]:
                        self.pod_node[pods[i]] = name
                    progress = True
            if not progress:
                return

    def node_claims(self):
        return list(self.launches)

    # ---- disruption --------------------------------------------------------------------------------------------------
    def cluster(self):
        """The disruption controller's snapshot (kpamd.model.Cluster) and the node names in its order."""
        from kpamd.model import Cluster, ClusterNode
        names = list(self.nodes)
        pods = [p for p in range(len(self.pod_shape)) if self.alive[p]]
        idx = {p: i for i, p in enumerate(pods)}
        existing, _ = self._existing(names)
        nodes = [ClusterNode(existing[e], 0, self.nodes[n]["type"], [idx[p] for p in self.pods_on(n)])
                 for e, n in enumerate(names)]
        cl = Cluster([self.types()], self.pools, nodes, self.shapes,
                     np.array([self.pod_shape[p] for p in pods], np.uint32),
                     np.array([self.pod_created[p] for p in pods], np.int64), np.array([p + 1 for p in pods], np.uint64),
                     name="e2e", pending=[idx[p] for p in pods if self.pod_node[p] is None],
                     spot_to_spot=self.spot_to_spot)
        return cl, names

    def _plan(self, cl):
        if self.backend == "device":
            import kpamd
            self.types()
            return kpamd.ClusterPlan(self.ctx, cl, catalogs=[self._cat])
        return OraclePlan(cl)

    def consolidate(self, max_commands=64):
        """The disruption controller until it finds nothing to do. Returns the commands applied."""
        from kpamd import disruption
        done = []
        for _ in range(max_commands):
            cl, names = self.cluster()
            plan = self._plan(cl)
            try:
                cmd = disruption.Controller().compute_command(cl, plan)
            finally:
                plan.close()
            if cmd is None:
                return done
            self._apply(cl, names, cmd)
            done.append(cmd)
            self.commands.append(cmd)
        raise AssertionError(f"consolidation did not settle after {max_commands} commands: {done[-4:]}")

    def _candidate_price(self, name):
        n = self.nodes[name]
        it = self.types()[n["type"]]
        return min(o.price for o in it.offerings if o.capacity_type == n["ct"] and o.zone == n["zone"]
                   and (o.reservation_id == n["rid"]))

    def _apply(self, cl, names, cmd):
        from kpamd import disruption
        cands = [names[c] for c in cmd.candidates]
        if cmd.method == "emptiness":
            for n in cands:
                del self.nodes[n]
            return
        moving = [p for n in cands for p in self.pods_on(n)] + self.pending()
        others = [n for n in names if n not in cands]
        res = self._solve(moving, others)
        new = None
        if cmd.decision == disruption.REPLACE:
            assert len(res["nodeclaims"]) == 1, res["nodeclaims"]
            nc = res["nodeclaims"][0]
            types = self.types()
            reqs = list(nc["requirements"])
            price = sum(self._candidate_price(n) for n in cands)
            s2s = all(self.nodes[n]["ct"] == "spot" for n in cands) and _has(reqs, CT, "spot")
            if s2s:  # the replacement launches spot only
                reqs = [r for r in reqs if r[0] != CT] + [(CT, "In", ["spot"])]
            opts = [t for t in nc["options"] if worst_launch_price(types[t], reqs, s2s) < price]
            if cmd.method == "multi":  # filterOutSameType
                same = {types[self.nodes[n]["type"]].name: self._candidate_price(n) for n in cands}
                mx = min([same[types[t].name] for t in opts if types[t].name in same] or [math.inf])
                opts = [t for t in opts if worst_launch_price(types[t], reqs, s2s) < mx]
            if s2s and len(cands) == 1:
                assert len(opts) >= 15, len(opts)
                opts = opts[:15]
            assert opts, "REPLACE without options"
            new = self._create(reqs, nc["requests"], opts, nc["nodepool"])
            assert new is not None, "replacement launch failed"
        for i, pl in enumerate(res["placement"]):
            pl = int(pl)
            if pl <= -2:
                self.pod_node[moving[i]] = others[-2 - pl]
            elif pl >= 0:
                self.pod_node[moving[i]] = new
            else:
                self.pod_node[moving[i]] = None
        for n in cands:
            del self.nodes[n]

    # ---- what the suites assert ------------------------------------------------------------------------------------
    def utilization(self, resource="cpu"):
        """Monitor.AvgUtilization (R:test/pkg/environment/common/monitor.go:201-234): the mean over Karpenter's nodes of
        requested / allocatable."""
        u = []
        for name in self.nodes:
            alloc = self.allocatable(name).get(resource, 0)
            if alloc:
                u.append(self._requested(self.pods_on(name)).get(resource, 0) / alloc)
        return sum(u) / len(u) if u else 0.0

    def type_of(self, name):
        return self.types()[self.nodes[name]["type"]].name

    def summary(self):
        """(type, zone, capacity type, reservation id, pod count) per node, in node order: the trajectory the device
        and the oracle must agree on."""
        return [(self.type_of(n), v["zone"], v["ct"], v["rid"], len(self.pods_on(n))) for n, v in self.nodes.items()]
