"""kpamd — Python host binding of the MI355X bin-packing hot path (libkp.so, include/kp/kp_abi.h).

The surfaces mirror the reference's plugin/operator interface for the path:
  CloudProvider.get_instance_types(nodepool)  <- R:pkg/cloudprovider/cloudprovider.go:177-193
  Scheduler(...).solve(pods)                  <- upstream scheduling.Scheduler.Solve
  compatible_available_filter(...)            <- R:pkg/providers/instance/filter/filter.go:39-64
  ClusterPlan(...).simulate(subsets)          <- upstream disruption computeConsolidation / SimulateScheduling
Everything computes behind the C ABI on the GPU; a missing libkp.so or HIP device raises.
"""
import ctypes as C
import os

import numpy as np

from . import abi
from .abi import Arena

_LIB = None
LIB_PATH = os.path.join(abi.PKG_ROOT, "libkp.so")


class KPError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"kp error {code}: {msg}")
        self.code = code


def load_lib(path=None):
    """Load libkp.so (built in-tree by __graft_entry__.build()). Raises if absent — no fallback."""
    global _LIB
    if _LIB is not None:
        return _LIB
    path = path or os.environ.get("KP_LIB") or LIB_PATH  # KP_LIB: a diagnostic build (tools/), same ABI
    if not os.path.exists(path):
        raise KPError(abi.KP_E_DEVICE, f"{path} missing: run __graft_entry__.build()")
    lib = C.CDLL(path)
    P = C.POINTER
    sig = {
        "kp_last_error": (C.c_char_p, []),
        "kp_abi_version": (C.c_int32, []),
        "kp_ctx_create": (C.c_int32, [P(abi.Options), P(C.c_void_p)]),
        "kp_ctx_destroy": (None, [C.c_void_p]),
        "kp_ctx_set_overrides": (C.c_int32, [C.c_void_p, P(abi.Overrides)]),
        "kp_ctx_get_overrides": (C.c_int32, [C.c_void_p, P(abi.Overrides)]),
        "kp_catalog_upload": (C.c_int32, [C.c_void_p, P(abi.CatalogDesc), C.c_uint64, P(C.c_void_p)]),
        "kp_catalog_seqnum": (C.c_uint64, [C.c_void_p]),
        "kp_catalog_size": (C.c_uint32, [C.c_void_p]),
        "kp_catalog_destroy": (None, [C.c_void_p]),
        "kp_catalog_update_offerings": (C.c_int32, [C.c_void_p, P(abi.OfferingUpdate), C.c_uint32, C.c_uint64]),
        "kp_instance_type_resolve": (C.c_int32, [P(abi.Options), P(abi.EC2Info), P(abi.NodeClass),
                                                 P(abi.ResourceList), P(abi.ResourceList)]),
        "kp_instance_type_overhead": (C.c_int32, [P(abi.Options), P(abi.EC2Info), P(abi.NodeClass),
                                                  P(abi.ResourceList), P(abi.ResourceList), P(abi.ResourceList)]),
        "kp_filter_compatible_available": (C.c_int32, [C.c_void_p, C.c_void_p, P(abi.FeasibilityQuery), C.c_uint32,
                                                       P(C.c_uint64), P(C.c_double), P(abi.SolveStats)]),
        "kp_filter_prepare": (C.c_int32, [C.c_void_p, C.c_void_p, P(abi.FeasibilityQuery), C.c_uint32, C.c_int32,
                                          P(C.c_void_p)]),
        "kp_filter_run": (C.c_int32, [C.c_void_p, P(C.c_uint64), P(C.c_double), P(abi.SolveStats)]),
        "kp_filter_run_compact": (C.c_int32, [C.c_void_p, P(C.c_uint64), P(C.c_uint64), P(abi.SolveStats)]),
        "kp_filter_class_prices": (C.c_int32, [C.c_void_p, P(C.c_double), C.c_uint32, P(C.c_uint32)]),
        "kp_filter_plan_destroy": (None, [C.c_void_p]),
        "kp_filter_refresh": (C.c_int32, [C.c_void_p, C.c_void_p]),
        "kp_launch_refresh": (C.c_int32, [C.c_void_p, C.c_void_p]),
        "kp_launch_prepare": (C.c_int32, [C.c_void_p, C.c_void_p, P(abi.LaunchRequest), C.c_uint32, P(C.c_char_p),
                                          C.c_uint32, C.c_uint32, P(C.c_void_p)]),
        "kp_launch_run": (C.c_int32, [C.c_void_p, P(abi.LaunchResult), P(C.c_uint32), P(C.c_uint32),
                                      P(abi.SolveStats)]),
        "kp_launch_plan_destroy": (None, [C.c_void_p]),
        "kp_launch_select": (C.c_int32, [C.c_void_p, C.c_void_p, P(abi.LaunchRequest), C.c_uint32, P(C.c_char_p),
                                         C.c_uint32, C.c_uint32, P(abi.LaunchResult), P(C.c_uint32), P(C.c_uint32),
                                         P(abi.SolveStats)]),
        "kp_solve": (C.c_int32, [C.c_void_p, P(abi.SolveIn), P(C.c_void_p)]),
        "kp_solve_validate": (C.c_int32, [P(abi.SolveIn)]),
        "kp_solve_prepare": (C.c_int32, [C.c_void_p, P(abi.SolveIn), P(C.c_void_p)]),
        "kp_solve_prepare_comm": (C.c_int32, [C.c_void_p, P(abi.SolveIn), C.c_void_p, P(C.c_void_p)]),
        "kp_solve_run": (C.c_int32, [C.c_void_p, P(C.c_void_p)]),
        "kp_solve_run_cancellable": (C.c_int32, [C.c_void_p, C.c_void_p, P(C.c_void_p)]),
        "kp_solve_cancellable": (C.c_int32, [C.c_void_p, P(abi.SolveIn), C.c_void_p, P(C.c_void_p)]),
        "kp_cancel_create": (C.c_int32, [C.c_void_p, P(C.c_void_p)]),
        "kp_cancel_set": (C.c_int32, [C.c_void_p]),
        "kp_cancel_reset": (C.c_int32, [C.c_void_p]),
        "kp_cancel_destroy": (None, [C.c_void_p]),
        "kp_solve_refresh": (C.c_int32, [C.c_void_p]),
        "kp_cluster_refresh": (C.c_int32, [C.c_void_p]),
        "kp_solve_plan_destroy": (None, [C.c_void_p]),
        "kp_result_nodeclaim_count": (C.c_uint32, [C.c_void_p]),
        "kp_result_pod_placements": (C.c_int32, [C.c_void_p, P(C.c_int32), C.c_uint32]),
        "kp_result_nodeclaim": (C.c_int32, [C.c_void_p, C.c_uint32, P(abi.NodeClaimInfo)]),
        "kp_result_stats": (C.c_int32, [C.c_void_p, P(abi.SolveStats)]),
        "kp_result_destroy": (None, [C.c_void_p]),
        "kp_simulate_batch": (C.c_int32, [C.c_void_p, P(abi.Cluster), P(C.c_uint32), P(C.c_uint32), C.c_uint32,
                                          C.c_int32, P(abi.SimResult), P(abi.SolveStats)]),
        "kp_cluster_prepare": (C.c_int32, [C.c_void_p, P(abi.Cluster), P(C.c_void_p)]),
        "kp_cluster_simulate": (C.c_int32, [C.c_void_p, P(C.c_uint32), P(C.c_uint32), C.c_uint32, C.c_int32,
                                            P(abi.SimResult), P(abi.SolveStats)]),
        "kp_cluster_simulate_cancellable": (C.c_int32, [C.c_void_p, C.c_void_p, P(C.c_uint32), P(C.c_uint32), C.c_uint32,
                                                        C.c_int32, P(abi.SimResult), P(abi.SolveStats)]),
        "kp_cluster_plan_destroy": (None, [C.c_void_p]),
        "kp_comm_unique_id": (C.c_int32, [C.c_char_p]),
        "kp_comm_init": (C.c_int32, [C.c_void_p, C.c_char_p, C.c_int32, C.c_int32, P(C.c_void_p)]),
        "kp_comm_destroy": (None, [C.c_void_p]),
        "kp_comm_init_all": (C.c_int32, [P(C.c_void_p), C.c_int32, P(C.c_void_p)]),
        "kp_comm_init_host": (C.c_int32, [C.c_void_p, C.c_int32, C.c_int32, abi.AllGatherFn, C.c_void_p,
                                          P(C.c_void_p)]),
        "kp_comm_rank": (C.c_int32, [C.c_void_p, P(C.c_int32), P(C.c_int32)]),
        "kp_consolidate_argmin": (C.c_int32, [C.c_void_p, C.c_void_p, P(C.c_uint32), P(C.c_uint32), C.c_uint32,
                                              C.c_uint64, C.c_int32, P(abi.SimResult), P(abi.Choice),
                                              P(abi.SolveStats)]),
        "kp_consolidate_argmin_cancellable": (C.c_int32, [C.c_void_p, C.c_void_p, C.c_void_p, P(C.c_uint32),
                                                          P(C.c_uint32), C.c_uint32, C.c_uint64, C.c_int32,
                                                          P(abi.SimResult), P(abi.Choice), P(abi.SolveStats)]),
        "kp_choice_reduce": (C.c_int32, [P(abi.Choice), C.c_uint32, P(abi.Choice)]),
    }
    for name, (res, args) in sig.items():
        f = getattr(lib, name, None)
        if f is None and path != LIB_PATH:  # a tools/ build of an older commit (A/B): its ABI may lack newer entries
            continue
        if f is None:
            raise KPError(abi.KP_E_DEVICE, f"{path} lacks {name}: rebuild (__graft_entry__.build())")
        f.restype = res
        f.argtypes = args
    _LIB = lib
    return lib


def _check(lib, rc):
    if rc != 0:
        raise KPError(rc, lib.kp_last_error().decode())


class Context:
    """kp_ctx: one HIP device + stream."""

    def __init__(self, device=0, vm_memory_overhead_percent=0.075, reserved_enis=0):
        self.lib = load_lib()
        self.opts = abi.Options(vm_memory_overhead_percent, reserved_enis, device)
        h = C.c_void_p()
        _check(self.lib, self.lib.kp_ctx_create(C.byref(self.opts), C.byref(h)))
        self.h = h

    def overrides(self):
        """kp_ctx_get_overrides -> dict of the kp_overrides fields."""
        ov = abi.Overrides()
        _check(self.lib, self.lib.kp_ctx_get_overrides(self.h, C.byref(ov)))
        return {k: getattr(ov, k) for k, _ in abi.Overrides._fields_}

    def set_overrides(self, **kw):
        """kp_ctx_set_overrides: the given kp_overrides fields, every other field 0 (the production choice)."""
        ov = abi.Overrides(**kw)
        _check(self.lib, self.lib.kp_ctx_set_overrides(self.h, C.byref(ov)))

    def close(self):
        if self.h:
            self.lib.kp_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Catalog:
    """A GetInstanceTypes result uploaded behind the ABI (kp_catalog_upload)."""

    def __init__(self, ctx, instance_types, seqnum=0):
        self.ctx = ctx
        self.instance_types = instance_types
        arena = Arena()
        desc = arena.catalog_desc(instance_types)
        h = C.c_void_p()
        _check(ctx.lib, ctx.lib.kp_catalog_upload(ctx.h, C.byref(desc), seqnum, C.byref(h)))
        self.h = h

    def update_offerings(self, updates, seqnum):
        """kp_catalog_update_offerings: UnavailableOfferings.MarkUnavailable + SeqNum bump
        (R:pkg/cache/unavailableofferings.go:66-92). updates: (type index, capacity type, zone, available[, price
        [, reservation id[, reservation capacity]]]); the matching offerings of self.instance_types change with the
        device-side catalogue (all or nothing)."""
        def opt(u, i):
            return u[i] if len(u) > i else None
        ups = [abi.OfferingUpdate(int(u[0]), 1 if u[3] else 0, u[1].encode() if u[1] is not None else None,
                                  u[2].encode() if u[2] is not None else None,
                                  float(u[4]) if opt(u, 4) is not None else float("nan"),
                                  opt(u, 5).encode() if opt(u, 5) is not None else None,
                                  int(opt(u, 6)) if opt(u, 6) is not None else -1, 0) for u in updates]
        arr = (abi.OfferingUpdate * max(1, len(ups)))(*ups)
        _check(self.ctx.lib, self.ctx.lib.kp_catalog_update_offerings(self.h, arr, len(ups), seqnum))
        for u in updates:
            for o in self.instance_types[u[0]].offerings:
                if o.capacity_type == u[1] and o.zone == u[2] and (opt(u, 5) is None or o.reservation_id == opt(u, 5)):
                    o.available = bool(u[3])
                    if opt(u, 4) is not None:
                        o.price = float(u[4])
                    if opt(u, 6) is not None and int(opt(u, 6)) >= 0:
                        o.reservation_capacity = int(opt(u, 6))

    def seqnum(self):
        return self.ctx.lib.kp_catalog_seqnum(self.h)

    def close(self):
        if self.h:
            self.ctx.lib.kp_catalog_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def validate(problem):
    """kp_solve_validate: host compile of the batch without a device (KP_OK or the error kp_solve would give)."""
    lib = load_lib()
    arena = Arena()
    handles = []
    for c in problem.catalogs:
        h = C.c_void_p()
        _check(lib, lib.kp_catalog_upload(None, C.byref(arena.catalog_desc(c)), 0, C.byref(h)))
        handles.append(h)
    try:
        si = abi.build_solve_in(arena, problem, catalog_handles=[h.value for h in handles])
        return lib.kp_solve_validate(C.byref(si))
    finally:
        for h in handles:
            lib.kp_catalog_destroy(h)


def read_result(lib, res, n_pods, prefix="kp_result_"):
    """Copy a (kp|kpo)_solve_result into plain Python: placement + NodeClaims in creation order."""
    get = lambda n: getattr(lib, prefix + n)
    placement = np.zeros(n_pods, dtype=np.int32)
    if n_pods:
        _check_generic(lib, get("pod_placements")(res, placement.ctypes.data_as(C.POINTER(C.c_int32)), n_pods))
    ncs = []
    n = get("nodeclaim_count")(res)
    for i in range(n):
        info = abi.NodeClaimInfo()
        _check_generic(lib, get("nodeclaim")(res, i, C.byref(info)))
        ncs.append({
            "nodepool": int(info.nodepool),
            "pods": [int(info.pods[j]) for j in range(info.n_pods)],
            "options": [int(info.options[j]) for j in range(info.n_options)],
            "n_remaining": int(info.n_remaining),
            "requirements": abi.read_requirements(info.requirements),
            "requests": abi.read_resources(info.requests),
        })
    st = abi.SolveStats()
    get("stats")(res, C.byref(st))
    return {"placement": placement, "nodeclaims": ncs, "stats": stats_dict(st)}


def stats_dict(st):
    d = {f: getattr(st, f) for f, _ in abi.SolveStats._fields_}
    d["phase_cycles"] = list(st.phase_cycles)
    d["attempt_cycles"] = list(st.attempt_cycles)
    d["fast_cycles"] = list(st.fast_cycles)
    d["fast_bails"] = list(st.fast_bails)
    d["order_chunks"] = list(st.order_chunks)
    return d


def _check_generic(lib, rc):
    if rc != 0:
        msg = lib.kp_last_error().decode() if hasattr(lib, "kp_last_error") else ""
        raise KPError(rc, msg)


class Scheduler:
    """upstream scheduling.Scheduler for one batch: NodePools (templates), existing nodes, catalogues."""

    def __init__(self, ctx, problem, catalogs=None):
        self.ctx = ctx
        self.problem = problem
        self.catalogs = catalogs or [Catalog(ctx, c) for c in problem.catalogs]

    def solve_in(self):
        """The kp_solve_in of this batch (marshalled once; the C ABI owns nothing of it)."""
        if getattr(self, "_si", None) is None:
            self._arena = Arena()
            self._si = abi.build_solve_in(self._arena, self.problem, catalog_handles=[c.h.value for c in self.catalogs])
        return self._si

    def solve(self, read=True):
        """kp_solve: compile the per-Solve half (the catalogue half comes resident from the ctx cache after the first
        Solve on these catalogues + NodePools), upload, run, copy the results back. read=False returns stats only."""
        lib = self.ctx.lib
        si = self.solve_in()
        res = C.c_void_p()
        _check(lib, lib.kp_solve(self.ctx.h, C.byref(si), C.byref(res)))
        try:
            if read:
                return read_result(lib, res, self.problem.n_pods)
            st = abi.SolveStats()
            lib.kp_result_stats(res, C.byref(st))
            return {"stats": stats_dict(st)}
        finally:
            lib.kp_result_destroy(res)

    def prepare(self, comm=None):
        """kp_solve_prepare: compile + upload once; returns a SolvePlan whose run() repeats Solve. With a Comm,
        kp_solve_prepare_comm: a collective whose template-options table is row-sharded over the ranks and
        all-gathered (every rank passes the same batch)."""
        return SolvePlan(self, comm)


class Cancel:
    """kp_cancel: the token a Go shim sets when ctx.Done() fires during a Solve (set() is lock-free, any thread)."""

    def __init__(self, ctx):
        self.ctx = ctx
        h = C.c_void_p()
        _check(ctx.lib, ctx.lib.kp_cancel_create(ctx.h, C.byref(h)))
        self.h = h

    def set(self):
        _check(self.ctx.lib, self.ctx.lib.kp_cancel_set(self.h))

    def reset(self):
        _check(self.ctx.lib, self.ctx.lib.kp_cancel_reset(self.h))

    def close(self):
        if self.h:
            self.ctx.lib.kp_cancel_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class SolvePlan:
    def __init__(self, sched, comm=None):
        self.sched = sched
        lib = sched.ctx.lib
        arena = Arena()
        si = abi.build_solve_in(arena, sched.problem, catalog_handles=[c.h.value for c in sched.catalogs])
        h = C.c_void_p()
        if comm is None:
            _check(lib, lib.kp_solve_prepare(sched.ctx.h, C.byref(si), C.byref(h)))
        else:
            _check(lib, lib.kp_solve_prepare_comm(sched.ctx.h, C.byref(si), comm.h, C.byref(h)))
        self.h = h

    def run(self, read=True, cancel=None):
        """kp_solve_run; with a Cancel token, kp_solve_run_cancellable (KPError KP_E_CANCELED once it is set)."""
        lib = self.sched.ctx.lib
        res = C.c_void_p()
        if cancel is None:
            _check(lib, lib.kp_solve_run(self.h, C.byref(res)))
        else:
            _check(lib, lib.kp_solve_run_cancellable(self.h, cancel.h, C.byref(res)))
        try:
            if read:
                return read_result(lib, res, self.sched.problem.n_pods)
            st = abi.SolveStats()
            lib.kp_result_stats(res, C.byref(st))
            return {"stats": stats_dict(st)}
        finally:
            lib.kp_result_destroy(res)

    def refresh(self):
        """kp_solve_refresh: re-apply the catalogues' current offerings (after update_offerings) in place."""
        _check(self.sched.ctx.lib, self.sched.ctx.lib.kp_solve_refresh(self.h))

    def close(self):
        if self.h:
            self.sched.ctx.lib.kp_solve_plan_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def compatible_available_filter(ctx, catalog, queries):
    """queries: list of (requirements, requests). Returns (kept bool[Q,T], cheapest f64[Q,T], stats)."""
    lib = ctx.lib
    arena = Arena()
    qs = arena.arr(abi.FeasibilityQuery, [abi.FeasibilityQuery(arena.requirements(r), arena.resources(q))
                                          for r, q in queries])
    T = len(catalog.instance_types)
    tiles = (T + 63) // 64
    mask = np.zeros(max(1, len(queries) * tiles), dtype=np.uint64)
    cheapest = np.zeros(max(1, len(queries) * T), dtype=np.float64)
    st = abi.SolveStats()
    _check(lib, lib.kp_filter_compatible_available(ctx.h, catalog.h, qs, len(queries),
                                                   mask.ctypes.data_as(C.POINTER(C.c_uint64)),
                                                   cheapest.ctypes.data_as(C.POINTER(C.c_double)), C.byref(st)))
    bits = np.unpackbits(mask[:len(queries) * tiles].view(np.uint8), bitorder="little").reshape(len(queries), tiles * 64)
    return bits[:, :T].astype(bool), cheapest[:len(queries) * T].reshape(len(queries), T), st


class FilterPlan:
    """kp_filter_prepare / kp_filter_run: CompatibleAvailableFilter rows resident on the device."""

    def __init__(self, ctx, catalog, queries, cheapest=True):
        """cheapest: True (KP_FILTER_CHEAPEST: a price row per query), False (mask only) or "compact"
        (KP_FILTER_COMPACT: the query's compatible offering classes; prices via class_prices())."""
        self.ctx = ctx
        self.T = len(catalog.instance_types)
        self.n = len(queries)
        mode = 2 if cheapest == "compact" else (1 if cheapest else 0)
        arena = Arena()
        qs = arena.arr(abi.FeasibilityQuery, [abi.FeasibilityQuery(arena.requirements(r), arena.resources(q))
                                              for r, q in queries])
        h = C.c_void_p()
        _check(ctx.lib, ctx.lib.kp_filter_prepare(ctx.h, catalog.h, qs, len(queries), mode, C.byref(h)))
        self.h = h

    def run(self, read=False):
        """One launch; read=True copies (kept bool[Q,T], cheapest f64[Q,T]) back, else results stay resident."""
        st = abi.SolveStats()
        lib = self.ctx.lib
        if not read:
            _check(lib, lib.kp_filter_run(self.h, None, None, C.byref(st)))
            return stats_dict(st)
        tiles = (self.T + 63) // 64
        mask = np.zeros(max(1, self.n * tiles), dtype=np.uint64)
        cheapest = np.zeros(max(1, self.n * self.T), dtype=np.float64)
        _check(lib, lib.kp_filter_run(self.h, mask.ctypes.data_as(C.POINTER(C.c_uint64)),
                                      cheapest.ctypes.data_as(C.POINTER(C.c_double)), C.byref(st)))
        bits = np.unpackbits(mask[:self.n * tiles].view(np.uint8), bitorder="little").reshape(self.n, tiles * 64)
        return bits[:, :self.T].astype(bool), cheapest[:self.n * self.T].reshape(self.n, self.T), stats_dict(st)

    def run_compact(self, read=True):
        """kp_filter_run_compact: (kept bool[Q,T], classes uint64[Q], stats); read=False: stats only."""
        st = abi.SolveStats()
        lib = self.ctx.lib
        if not read:
            _check(lib, lib.kp_filter_run_compact(self.h, None, None, C.byref(st)))
            return stats_dict(st)
        tiles = (self.T + 63) // 64
        mask = np.zeros(max(1, self.n * tiles), dtype=np.uint64)
        cls = np.zeros(max(1, self.n), dtype=np.uint64)
        _check(lib, lib.kp_filter_run_compact(self.h, mask.ctypes.data_as(C.POINTER(C.c_uint64)),
                                              cls.ctypes.data_as(C.POINTER(C.c_uint64)), C.byref(st)))
        bits = np.unpackbits(mask[:self.n * tiles].view(np.uint8), bitorder="little").reshape(self.n, tiles * 64)
        return bits[:, :self.T].astype(bool), cls[:self.n], stats_dict(st)

    def class_prices(self):
        """kp_filter_class_prices: float64[C, T], the cheapest available offering of each type per offering class."""
        lib = self.ctx.lib
        n = C.c_uint32()
        _check(lib, lib.kp_filter_class_prices(self.h, None, 0, C.byref(n)))
        out = np.zeros(max(1, n.value * self.T), dtype=np.float64)
        _check(lib, lib.kp_filter_class_prices(self.h, out.ctypes.data_as(C.POINTER(C.c_double)), out.size,
                                               C.byref(n)))
        return out[:n.value * self.T].reshape(n.value, self.T)

    @staticmethod
    def cheapest_from_compact(classes, class_prices):
        """min over the row's classes of the class price rows (+inf: none) = kp_filter_run's out_cheapest."""
        out = np.full((len(classes), class_prices.shape[1]), np.inf)
        for c in range(class_prices.shape[0]):
            sel = ((classes >> np.uint64(c)) & np.uint64(1)).astype(bool)
            out[sel] = np.minimum(out[sel], class_prices[c])
        return out

    def refresh(self, catalog):
        """kp_filter_refresh: re-apply the catalogue's current offerings (ICE / price) to the resident plan."""
        _check(self.ctx.lib, self.ctx.lib.kp_filter_refresh(self.h, catalog.h))

    def close(self):
        if self.h:
            self.ctx.lib.kp_filter_plan_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


MAX_LAUNCH_TYPES = 60  # maxInstanceTypes (R:pkg/providers/instance/instance.go:60)


class LaunchPlan:
    """kp_launch_prepare / kp_launch_run: instance.DefaultProvider.Create's launch-side selection for a batch of
    NodeClaims (filters, Truncate, capacity type, CreateFleet overrides), requests resident on the device.
    requests: [(requirements, requests, [catalogue indices])]; subnet_zones: zones with a launch subnet."""

    def __init__(self, ctx, catalog, requests, subnet_zones, max_types=MAX_LAUNCH_TYPES):
        self.ctx = ctx
        self.n = len(requests)
        self.zones = list(subnet_zones)
        self.max_types = max_types
        arena = Arena()
        rq = abi.launch_requests(arena, requests)
        zs = arena.arr(C.c_char_p, [z.encode() for z in self.zones])
        h = C.c_void_p()
        _check(ctx.lib, ctx.lib.kp_launch_prepare(ctx.h, catalog.h, rq, self.n, zs, len(self.zones), max_types,
                                                  C.byref(h)))
        self.h = h

    def run(self, read=True):
        """One launch; read=True returns ([result dict per request], stats), else (None, stats)."""
        st = abi.SolveStats()
        lib = self.ctx.lib
        if not read:
            _check(lib, lib.kp_launch_run(self.h, None, None, None, C.byref(st)))
            return None, stats_dict(st)
        out = (abi.LaunchResult * max(1, self.n))()
        stride = self.max_types * max(1, len(self.zones))
        types = np.zeros(max(1, self.n * self.max_types), dtype=np.uint32)
        ovr = np.zeros(max(1, self.n * stride), dtype=np.uint32)
        _check(lib, lib.kp_launch_run(self.h, out, types.ctypes.data_as(C.POINTER(C.c_uint32)),
                                      ovr.ctypes.data_as(C.POINTER(C.c_uint32)), C.byref(st)))
        res = [abi.launch_result_dict(out[i], types[i * self.max_types:(i + 1) * self.max_types],
                                      ovr[i * stride:(i + 1) * stride], self.zones) for i in range(self.n)]
        return res, stats_dict(st)

    def refresh(self, catalog):
        """kp_launch_refresh: re-apply the catalogue's current offerings (ICE / price) to the resident plan."""
        _check(self.ctx.lib, self.ctx.lib.kp_launch_refresh(self.h, catalog.h))

    def close(self):
        if self.h:
            self.ctx.lib.kp_launch_plan_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def launch_requests_from_solve(result):
    """One launch request per NodeClaim of a Solve result: its final requirements, requests and options."""
    reqs = []
    for n in result["nodeclaims"]:
        reqs.append((n["requirements"], n["requests"], n["options"]))
    return reqs


def pod_queries(problem):
    """One CompatibleAvailableFilter row per pod: NewPodRequirements (nodeSelector + heaviest preferred term +
    first required term) and the pod's requests."""
    rows = []
    for sh in problem.shapes:
        reqs = [(k, "In", [v]) for k, v in sh.node_selector.items()]
        if sh.preferred_terms:
            reqs += list(max(sh.preferred_terms, key=lambda t: t[0])[1])
        if sh.required_terms:
            reqs += list(sh.required_terms[0])
        rows.append((reqs, sh.requests))
    return [rows[int(s)] for s in problem.pod_shape]


def sim_dict(r):
    """kp_sim_result (ctypes struct or a record of abi.sim_dtype()) -> dict."""
    if isinstance(r, np.void):
        g, np_key = (lambda k: r[k]), "nodepool"
    else:
        g, np_key = (lambda k: getattr(r, k)), "replacement_nodepool"
    return {"decision": int(g("decision")), "nodepool": int(g(np_key)),
            "candidate_price": float(g("candidate_price")), "replacement_price": float(g("replacement_price")),
            "savings": float(g("savings")), "n_options": int(g("n_options")), "n_pods": int(g("n_pods"))}


class ClusterPlan:
    """Resident cluster snapshot for consolidation (kp_cluster_prepare); simulate() evaluates a batch of
    candidate subsets as computeConsolidation would (kp_cluster_simulate)."""

    def __init__(self, ctx, cluster, catalogs=None):
        import time
        self.ctx = ctx
        self.cluster = cluster
        t0 = time.perf_counter()
        self.catalogs = catalogs or [Catalog(ctx, c) for c in cluster.catalogs]
        t1 = time.perf_counter()
        arena = Arena()
        cl = abi.build_cluster(arena, cluster, catalog_handles=[c.h.value for c in self.catalogs])
        t2 = time.perf_counter()
        h = C.c_void_p()
        _check(ctx.lib, ctx.lib.kp_cluster_prepare(ctx.h, C.byref(cl), C.byref(h)))
        self.h = h
        # where the construction's time went: catalogue upload (when not passed in), this binding's marshalling of the
        # cluster into kp_cluster structs (a caller's shim builds those itself), and kp_cluster_prepare
        self.prepare_times = {"catalog_s": t1 - t0, "marshal_s": t2 - t1, "kp_cluster_prepare_s": time.perf_counter() - t2}

    def refresh(self):
        """kp_cluster_refresh: re-apply the catalogues' current offerings (after update_offerings) in place."""
        _check(self.ctx.lib, self.ctx.lib.kp_cluster_refresh(self.h))

    def simulate(self, subsets, multi_node=True, raw=False, cancel=None):
        """subsets: list of node-index lists (candidate order). Returns (results, stats); raw=True returns
        the kp_sim_result array instead of dicts. cancel: a Cancel token (kp_cluster_simulate_cancellable)."""
        arena = Arena()
        offs, flat = abi.subsets_csr(arena, subsets)
        out = (abi.SimResult * max(1, len(subsets)))()
        st = abi.SolveStats()
        _check(self.ctx.lib, self.ctx.lib.kp_cluster_simulate_cancellable(
            self.h, cancel.h if cancel is not None else None, offs, flat, len(subsets), 1 if multi_node else 0,
            out, C.byref(st)))
        if raw:
            return out, stats_dict(st)
        return [sim_dict(out[i]) for i in range(len(subsets))], stats_dict(st)

    def simulate_csr(self, offsets, nodes, multi_node=True, cancel=None):
        """CSR batch (uint32 offsets[n+1], node indices) -> numpy structured array (abi.sim_dtype()), stats."""
        offsets = np.ascontiguousarray(offsets, dtype=np.uint32)
        nodes = np.ascontiguousarray(nodes, dtype=np.uint32)
        n = len(offsets) - 1
        out = np.zeros(max(n, 1), dtype=abi.sim_dtype())
        st = abi.SolveStats()
        P = C.POINTER
        _check(self.ctx.lib, self.ctx.lib.kp_cluster_simulate_cancellable(
            self.h, cancel.h if cancel is not None else None, offsets.ctypes.data_as(P(C.c_uint32)), nodes.ctypes.data_as(P(C.c_uint32)) if len(nodes) else None,
            n, 1 if multi_node else 0, out.ctypes.data_as(P(abi.SimResult)), C.byref(st)))
        return out[:n], stats_dict(st)

    def argmin(self, offsets, nodes, base_index=0, comm=None, multi_node=True, read_all=False, cancel=None):
        """kp_consolidate_argmin: this rank's subsets (CSR, global indices base_index + i) simulated, reduced on the
        device and across ranks (RCCL all-gather when comm is a Comm). Returns (choice dict, per-subset results
        or None, stats). cancel: a Cancel token (kp_consolidate_argmin_cancellable)."""
        offsets = np.ascontiguousarray(offsets, dtype=np.uint32)
        nodes = np.ascontiguousarray(nodes, dtype=np.uint32)
        n = len(offsets) - 1
        out = np.zeros(max(n, 1), dtype=abi.sim_dtype()) if read_all else None
        ch = abi.Choice()
        st = abi.SolveStats()
        P = C.POINTER
        _check(self.ctx.lib, self.ctx.lib.kp_consolidate_argmin_cancellable(
            self.h, comm.h if comm is not None else None, cancel.h if cancel is not None else None,
            offsets.ctypes.data_as(P(C.c_uint32)),
            nodes.ctypes.data_as(P(C.c_uint32)) if len(nodes) else None, n, int(base_index), 1 if multi_node else 0,
            out.ctypes.data_as(P(abi.SimResult)) if out is not None else None, C.byref(ch), C.byref(st)))
        return choice_dict(ch), (out[:n] if out is not None else None), stats_dict(st)

    def close(self):
        if self.h:
            self.ctx.lib.kp_cluster_plan_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def choice_dict(ch):
    return {"subset": int(ch.subset), "counts": [int(x) for x in ch.counts], "overflowed": int(ch.overflowed),
            "result": sim_dict(ch.result)}


def comm_unique_id(lib=None):
    """kp_comm_unique_id (rank 0): 128 bytes every rank passes to Comm."""
    lib = lib or load_lib()
    buf = C.create_string_buffer(abi.COMM_ID_BYTES)
    _check(lib, lib.kp_comm_unique_id(buf))
    return buf.raw


class Comm:
    """kp_comm: one rank of a communicator over the node's GPUs. Comm(ctx, uid, n, rank) is one rank of an RCCL
    communicator (kp_comm_init, collective, one process per GPU); Comm.init_all(ctxs) builds the n RCCL ranks of one
    process (kp_comm_init_all, one thread per GPU); Comm.host(ctx, n, rank, allgather) uses a host all-gather
    (kp_comm_init_host): allgather(rank, data: bytes) -> list of n bytes objects, blocking until every rank sent."""

    def __init__(self, ctx, uid=None, n_ranks=1, rank=0, _handle=None):
        self.ctx = ctx
        self._cb = None
        if _handle is not None:
            self.h = _handle
            return
        h = C.c_void_p()
        _check(ctx.lib, ctx.lib.kp_comm_init(ctx.h, bytes(uid), n_ranks, rank, C.byref(h)))
        self.h = h

    @classmethod
    def init_all(cls, ctxs):
        lib = ctxs[0].lib
        hs = (C.c_void_p * len(ctxs))(*[c.h for c in ctxs])
        out = (C.c_void_p * len(ctxs))()
        _check(lib, lib.kp_comm_init_all(hs, len(ctxs), out))
        return [cls(c, _handle=C.c_void_p(out[i])) for i, c in enumerate(ctxs)]

    @classmethod
    def host(cls, ctx, n_ranks, rank, allgather):
        def fn(_user, r, send, recv, nbytes):
            try:
                parts = allgather(int(r), C.string_at(send, nbytes))
                C.memmove(recv, b"".join(parts), nbytes * n_ranks)
                return 0
            except Exception:  # the library turns a non-zero return into KP_E_DEVICE
                return 1
        cb = abi.AllGatherFn(fn)
        h = C.c_void_p()
        _check(ctx.lib, ctx.lib.kp_comm_init_host(ctx.h, n_ranks, rank, cb, None, C.byref(h)))
        c = cls(ctx, _handle=h)
        c._cb = cb  # keep the trampoline alive as long as the communicator
        return c

    def rank(self):
        r, n = C.c_int32(), C.c_int32()
        _check(self.ctx.lib, self.ctx.lib.kp_comm_rank(self.h, C.byref(r), C.byref(n)))
        return r.value, n.value

    def close(self):
        if self.h:
            self.ctx.lib.kp_comm_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class ThreadAllGather:
    """In-process host all-gather for n threads (one per kp_ctx): the exchange step of Comm.host when the ranks
    are threads of one process (the one-goroutine-per-GPU pattern; tests run it on one GPU)."""

    def __init__(self, n):
        import threading
        self.n = n
        self.slots = [None] * n
        self.b1 = threading.Barrier(n)
        self.b2 = threading.Barrier(n)

    def __call__(self, rank, data):
        self.slots[rank] = data
        self.b1.wait(timeout=120)
        out = list(self.slots)
        self.b2.wait(timeout=120)
        return out


def torch_allgather(group=None):
    """Host all-gather over torch.distributed (e.g. gloo across processes) for Comm.host."""
    import torch
    import torch.distributed as dist

    def ag(rank, data):
        n = dist.get_world_size(group)
        t = torch.frombuffer(bytearray(data), dtype=torch.uint8)
        parts = [torch.empty_like(t) for _ in range(n)]
        dist.all_gather(parts, t, group=group)
        return [bytes(p.numpy().tobytes()) for p in parts]
    return ag


def choice_reduce(records, lib=None):
    """kp_choice_reduce over per-rank kp_choice records (the all-gather's host step)."""
    lib = lib or load_lib()
    arr = (abi.Choice * max(1, len(records)))(*records)
    out = abi.Choice()
    _check(lib, lib.kp_choice_reduce(arr, len(records), C.byref(out)))
    return out
