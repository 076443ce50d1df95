"""Disruption-side callers of the batched simulation (kp_cluster_simulate), mirroring upstream
pkg/controllers/disruption (sigs.k8s.io/karpenter v1.5.1, absent from the container; behaviour per SURVEY §3
CS3 and R:website/content/en/preview/concepts/disruption.md:89-128):

  SingleNodeConsolidation.compute_command   the first candidate (disruption-cost order) whose
                                            computeConsolidation is not a no-op
  MultiNodeConsolidation.first_n_option     firstNConsolidationOption's binary search over prefixes
                                            candidates[0:mid+1], lo=1, hi = len-1 if len <= 100 else 100
                                            (ComputeCommand passes max = Clamp(len, 0, MaxParallel=100) and
                                            firstN lowers it to len-1 only when len <= max); every prefix
                                            the search can touch is simulated in ONE batch, then the
                                            search is replayed exactly over those results
  sweep(...)                                the config-4 sweep: this rank's contiguous share of the subsets
                                            through kp_consolidate_argmin (simulation, device argmax, one
                                            RCCL all-gather of the ranks' records inside libkp)
  local_choice(...)                         a rank's kp_choice record from per-subset results on the host
                                            (what the device argmax produces; CPU tests and other transports)
  Emptiness.compute_command                 the candidates without reschedulable pods, deleted in one command
  candidate_order(cluster)                  the consolidatable nodes in disruption-cost order (ReschedulingCost of
                                            default-priority pods = their count; ties by node name)
  Controller.compute_command(cluster, plan) one disruption pass over the methods the e2e consolidation suite
                                            exercises, in upstream order (Emptiness, MultiNodeConsolidation,
                                            SingleNodeConsolidation): the first method that returns a command wins

Decisions are kp_decision values: 0 no-op, 1 delete, 2 replace.
"""
import numpy as np

NOOP, DELETE, REPLACE = 0, 1, 2


class Command:
    """A disruption command: the method that produced it, its candidates (cluster node indices, candidate order), the
    decision (DELETE / REPLACE) and the computeConsolidation result (savings, replacement NodePool and price, ...)."""

    def __init__(self, method, candidates, decision, result=None):
        self.method = method
        self.candidates = list(candidates)
        self.decision = decision
        self.result = result or {}

    def __repr__(self):
        return f"Command({self.method}, {self.candidates}, {('noop', 'delete', 'replace')[self.decision]})"


def candidate_order(cluster, nodes=None):
    """Consolidation candidates in disruption-cost order (R:website/content/en/preview/concepts/disruption.md:101-103:
    the candidates that are cheapest to disrupt first). Every pod here has the default priority and deletion cost, so
    ReschedulingCost is the pod count; nodes marked for deletion are never candidates; ties go by node name (upstream
    sorts a slice built from a map: parity unpinned)."""
    idx = [i for i in (range(len(cluster.nodes)) if nodes is None else nodes) if not cluster.nodes[i].deleting]
    return sorted(idx, key=lambda i: (len(cluster.nodes[i].pods), cluster.nodes[i].node.name))


class Emptiness:
    """Emptiness (WhenEmptyOrUnderutilized with consolidateAfter elapsed): every candidate node without reschedulable
    pods is deleted, all in one command (disruption budgets are not modelled: 100 %)."""

    def compute_command(self, cluster, candidates):
        empty = [c for c in candidates if not cluster.nodes[c].pods]
        return Command("emptiness", empty, DELETE, {"decision": DELETE}) if empty else None


class Controller:
    """One pass of the disruption controller over the consolidation methods, in upstream order: Emptiness, then
    MultiNodeConsolidation (firstNConsolidationOption over the disruption-cost order), then SingleNodeConsolidation
    (the first candidate whose computeConsolidation is not a no-op). plan: the resident snapshot of `cluster`
    (ClusterPlan, or any object with the same simulate(subsets, multi_node))."""

    def compute_command(self, cluster, plan):
        cands = candidate_order(cluster)
        cmd = Emptiness().compute_command(cluster, cands)
        if cmd is not None:
            return cmd
        cands = [c for c in cands if cluster.nodes[c].pods]
        hit = MultiNodeConsolidation(plan).first_n_option(cands)
        if hit is not None:
            n, r = hit
            return Command("multi", cands[:n], r["decision"], r)
        hit = SingleNodeConsolidation(plan).compute_command(cands)
        if hit is not None:
            c, r = hit
            return Command("single", [c], r["decision"], r)
        return None


class SingleNodeConsolidation:
    def __init__(self, plan):
        self.plan = plan

    def compute_command(self, candidates):
        """Returns (candidate, result) of the first candidate whose simulation is not a no-op, or None."""
        if not candidates:
            return None
        res, _ = self.plan.simulate([[c] for c in candidates], multi_node=False)
        for c, r in zip(candidates, res):
            if r["decision"] != NOOP:
                return c, r
        return None


class MultiNodeConsolidation:
    MAX_PARALLEL = 100  # upstream MultiNodeConsolidation MaxParallel

    def __init__(self, plan):
        self.plan = plan

    @staticmethod
    def search_hi(n):
        """firstNConsolidationOption's initial max: ComputeCommand passes Clamp(n, 0, 100); if n <= max it becomes
        n - 1 (so with more than 100 candidates the search can reach the 101-candidate prefix)."""
        mx = min(max(n, 0), MultiNodeConsolidation.MAX_PARALLEL)
        return n - 1 if n <= mx else mx

    @staticmethod
    def search_prefixes(n):
        """Every mid the binary search can evaluate (prefix length mid+1)."""
        if n < 2:
            return []
        return list(range(1, MultiNodeConsolidation.search_hi(n) + 1))

    @staticmethod
    def replay(n, results_by_mid):
        """firstNConsolidationOption over precomputed computeConsolidation(candidates[0:mid+1]) results."""
        if n < 2:
            return None
        lo, hi = 1, MultiNodeConsolidation.search_hi(n)
        best = None
        while lo <= hi:
            mid = (lo + hi) // 2
            r = results_by_mid[mid]
            if r["decision"] == DELETE or (r["decision"] == REPLACE and r["n_options"] > 0):
                best = (mid, r)
                lo = mid + 1
            else:
                hi = mid - 1
        return best

    def first_n_option(self, candidates):
        """Returns (prefix length, result) of the command firstNConsolidationOption picks, or None."""
        mids = self.search_prefixes(len(candidates))
        if not mids:
            return None
        res, _ = self.plan.simulate([candidates[:m + 1] for m in mids], multi_node=True)
        by_mid = dict(zip(mids, res))
        hit = self.replay(len(candidates), by_mid)
        return None if hit is None else (hit[0] + 1, hit[1])


def random_subsets_csr(n_candidates, n_subsets, seed, max_size=100, min_size=2):
    """n_subsets random subsets of candidate POSITIONS (2..max_size each, distinct, ascending), CSR."""
    rng = np.random.default_rng(seed)
    k = rng.integers(min_size, min(max_size, n_candidates) + 1, size=n_subsets)
    picks = rng.integers(0, n_candidates, size=(n_subsets, int(k.max())))
    picks = np.sort(np.where(np.arange(picks.shape[1])[None, :] < k[:, None], picks, np.iinfo(np.int64).max), axis=1)
    valid = picks != np.iinfo(np.int64).max
    valid[:, 1:] &= picks[:, 1:] != picks[:, :-1]  # drop repeats: subsets stay sets
    sizes = valid.sum(axis=1)
    offs = np.zeros(n_subsets + 1, dtype=np.uint32)
    offs[1:] = np.cumsum(sizes)
    return offs, picks[valid].astype(np.uint32)


SWEEP_CHUNK = 1 << 16  # subsets per generation chunk of the config-4 sweep (chunk c uses seed 1000 + c)


def sweep_subsets(candidates, n_subsets, chunk_lo=0, chunk_hi=None):
    """The config-4 sweep's random candidate subsets (2..100 candidates each), chunks [chunk_lo, chunk_hi) of
    SWEEP_CHUNK subsets concatenated into one CSR over cluster node indices; the set does not depend on how the
    chunks are split over ranks. Returns (offsets, nodes, global index of the first subset)."""
    cands = np.asarray(candidates, dtype=np.uint32)
    n_chunks = (n_subsets + SWEEP_CHUNK - 1) // SWEEP_CHUNK
    chunk_hi = n_chunks if chunk_hi is None else chunk_hi
    offs_l, nodes_l, base = [], [], 0
    for c in range(chunk_lo, chunk_hi):
        n = min(SWEEP_CHUNK, n_subsets - c * SWEEP_CHUNK)
        offs, pos = random_subsets_csr(len(cands), n, seed=1000 + c)
        offs_l.append(offs[:-1] + base)
        nodes_l.append(cands[pos])
        base += int(offs[-1])
    offs_l.append(np.array([base], dtype=np.uint32))
    return (np.concatenate(offs_l).astype(np.uint32),
            np.concatenate(nodes_l) if nodes_l else np.zeros(0, dtype=np.uint32), chunk_lo * SWEEP_CHUNK)


def best_local(results, base_index=0):
    """(savings, global subset index) of the best non-no-op decision in this shard; (-inf, -1) if none."""
    dec = np.array([int(r.decision) for r in results], dtype=np.int32) if not isinstance(results, np.ndarray) else results["decision"]
    sav = np.array([r.savings for r in results], dtype=np.float64) if not isinstance(results, np.ndarray) else results["savings"]
    sav = np.where(dec != NOOP, sav, -np.inf)
    if len(sav) == 0 or not np.isfinite(sav.max()):
        return -np.inf, -1
    i = int(np.argmax(sav))  # first index of the max: ties -> lowest subset index
    return float(sav[i]), base_index + i


def reduce_best(savings, index, dist=None, device=None):
    """Cross-rank argmax of (savings, -index) as two scalar all-reduces (RCCL over xGMI on the GPU path):
    MAX of the savings, then MIN of the subset index among the ranks holding that maximum. Exact (no packing of
    the f64 savings into a key) and deterministic: ties go to the lowest global subset index."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return savings, index
    import torch
    s = torch.tensor([savings if index >= 0 else -np.inf], dtype=torch.float64, device=device)
    dist.all_reduce(s, op=dist.ReduceOp.MAX)
    best_s = float(s.item())
    if not np.isfinite(best_s):
        return -np.inf, -1
    mine = index >= 0 and savings == best_s
    i = torch.tensor([index if mine else np.iinfo(np.int64).max], dtype=torch.int64, device=device)
    dist.all_reduce(i, op=dist.ReduceOp.MIN)
    return best_s, int(i.item())


def shard(n, rank, world):
    """Contiguous block of [0, n) for this rank."""
    per = (n + world - 1) // world
    lo = min(n, rank * per)
    return lo, min(n, lo + per)


def local_choice(results, base_index=0):
    """kp_choice record of one rank from its per-subset results (dicts or the simulate_csr structured array): the
    best non-no-op decision (savings desc, global subset index asc) and the decision counts."""
    from . import abi
    ch = abi.Choice()
    ch.subset = -1
    dec = [int(r["decision"]) for r in results]
    for k in range(3):
        ch.counts[k] = sum(1 for d in dec if d == k)
    s, i = best_local(results if isinstance(results, np.ndarray) else _as_struct(results), base_index)
    if i >= 0:
        r = results[i - base_index]
        ch.subset = i
        ch.result = abi.SimResult(int(r["decision"]), int(r["nodepool"]), float(r["candidate_price"]),
                                  float(r["replacement_price"]), float(r["savings"]), int(r["n_options"]),
                                  int(r["n_pods"]))
    return ch


def _as_struct(results):
    from . import abi
    out = np.zeros(len(results), dtype=abi.sim_dtype())
    for j, r in enumerate(results):
        out[j]["decision"] = r["decision"]
        out[j]["savings"] = r["savings"]
    return out


def sweep(plan, offsets, nodes, base_index=0, comm=None, multi_node=True):
    """The config-4 sweep step of one rank: kp_consolidate_argmin over this rank's CSR subsets (global indices
    base_index + i); with a Comm the best decision is reduced across ranks inside libkp (RCCL all-gather).
    Returns (choice, stats)."""
    ch, _, st = plan.argmin(offsets, nodes, base_index=base_index, comm=comm, multi_node=multi_node)
    return ch, st
