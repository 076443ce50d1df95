"""ctypes loader for oracle/liboracle.so — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module (as the
checker / the timed CPU baseline). The product package never imports it.
"""
import ctypes as C
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(REPO, "karpenter-provider-aws_amd"))
from kpamd import abi  # noqa: E402  (struct layouts only: the shared ABI, not product code paths)

LIB_PATH = os.path.join(HERE, "liboracle.so")
_LIB = None


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


def load(path=LIB_PATH):
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(path):
        build()
    lib = C.CDLL(path)
    P = C.POINTER
    sig = {
        "kpo_solve": (C.c_int32, [P(abi.SolveIn), P(C.c_void_p)]),
        "kpo_result_nodeclaim_count": (C.c_uint32, [C.c_void_p]),
        "kpo_result_pod_placements": (C.c_int32, [C.c_void_p, P(C.c_int32), C.c_uint32]),
        "kpo_result_nodeclaim": (C.c_int32, [C.c_void_p, C.c_uint32, P(abi.NodeClaimInfo)]),
        "kpo_result_stats": (C.c_int32, [C.c_void_p, P(abi.SolveStats)]),
        "kpo_result_destroy": (None, [C.c_void_p]),
        "kpo_filter_compatible_available": (C.c_int32, [P(abi.CatalogDesc), P(abi.FeasibilityQuery), P(C.c_uint8),
                                                        P(C.c_double)]),
        "kpo_filter_spot": (C.c_int32, [P(abi.CatalogDesc), P(abi.Requirements), P(C.c_uint8)]),
        "kpo_launch_select": (C.c_int32, [P(abi.CatalogDesc), P(abi.LaunchRequest), P(C.c_char_p), C.c_uint32,
                                          C.c_uint32, P(abi.LaunchResult), P(C.c_uint32), P(C.c_uint32)]),
        "kpo_filter_exotic": (C.c_int32, [P(abi.CatalogDesc), P(abi.Requirements), P(C.c_uint8)]),
        "kpo_filter_reservation": (C.c_int32, [P(abi.CatalogDesc), P(abi.Requirements), C.c_int32, P(C.c_uint8),
                                               P(C.c_uint8)]),
        "kpo_requirements_compatible": (C.c_int32, [P(abi.Requirements), P(abi.Requirements), C.c_int32]),
        "kpo_requirements_intersects": (C.c_int32, [P(abi.Requirements), P(abi.Requirements)]),
        "kpo_instance_type_resolve": (C.c_int32, [P(abi.Options), P(abi.EC2Info), P(abi.NodeClass),
                                                  P(abi.ResourceList), C.c_void_p]),
        "kpo_simulate_batch": (C.c_int32, [P(abi.Cluster), P(C.c_uint32), P(C.c_uint32), C.c_uint32, C.c_int32,
                                           P(abi.SimResult), P(abi.SolveStats)]),
    }
    for name, (res, args) in sig.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    _LIB = lib
    return lib


class Overhead(C.Structure):
    _fields_ = [("kube_reserved", abi.ResourceList), ("system_reserved", abi.ResourceList),
                ("eviction_threshold", abi.ResourceList)]


def solve(problem):
    """Oracle Scheduler.Solve + TruncateInstanceTypes over the same inputs the device path takes."""
    from kpamd import read_result
    lib = load()
    arena = abi.Arena()
    si = abi.build_solve_in(arena, problem, catalog_handles=None)
    res = C.c_void_p()
    rc = lib.kpo_solve(C.byref(si), C.byref(res))
    if rc != 0:
        raise RuntimeError(f"kpo_solve = {rc}")
    try:
        return read_result(lib, res, problem.n_pods, prefix="kpo_result_")
    finally:
        lib.kpo_result_destroy(res)


def compatible_available_filter(instance_types, requirements, requests):
    lib = load()
    arena = abi.Arena()
    desc = arena.catalog_desc(instance_types)
    q = abi.FeasibilityQuery(arena.requirements(requirements), arena.resources(requests))
    kept = np.zeros(max(1, len(instance_types)), dtype=np.uint8)
    cheapest = np.zeros(max(1, len(instance_types)), dtype=np.float64)
    lib.kpo_filter_compatible_available(C.byref(desc), C.byref(q), kept.ctypes.data_as(C.POINTER(C.c_uint8)),
                                        cheapest.ctypes.data_as(C.POINTER(C.c_double)))
    return kept[:len(instance_types)].astype(bool), cheapest[:len(instance_types)]


def _filter(fn, instance_types, requirements):
    lib = load()
    arena = abi.Arena()
    desc = arena.catalog_desc(instance_types)
    reqs = arena.requirements(requirements)
    kept = np.zeros(max(1, len(instance_types)), dtype=np.uint8)
    getattr(lib, fn)(C.byref(desc), C.byref(reqs), kept.ctypes.data_as(C.POINTER(C.c_uint8)))
    return kept[:len(instance_types)].astype(bool)


def spot_filter(instance_types, requirements):
    return _filter("kpo_filter_spot", instance_types, requirements)


def exotic_filter(instance_types, requirements):
    return _filter("kpo_filter_exotic", instance_types, requirements)


def reservation_filter(instance_types, requirements, which):
    """CapacityReservationType ("type") / CapacityBlock ("block") / ReservedOffering ("offering") filter:
    (kept type flags, per type the indices of its offerings in the replaced slice)."""
    lib = load()
    arena = abi.Arena()
    desc = arena.catalog_desc(instance_types)
    reqs = arena.requirements(requirements)
    n_off = sum(len(t.offerings) for t in instance_types)
    kept = np.zeros(max(1, len(instance_types)), dtype=np.uint8)
    okept = np.zeros(max(1, n_off), dtype=np.uint8)
    rc = lib.kpo_filter_reservation(C.byref(desc), C.byref(reqs), {"type": 0, "block": 1, "offering": 2}[which],
                                    kept.ctypes.data_as(C.POINTER(C.c_uint8)), okept.ctypes.data_as(C.POINTER(C.c_uint8)))
    if rc != 0:
        raise RuntimeError(f"kpo_filter_reservation = {rc}")
    offs, i = [], 0
    for t in instance_types:
        offs.append([j for j in range(len(t.offerings)) if okept[i + j]])
        i += len(t.offerings)
    return kept[:len(instance_types)].astype(bool), offs


def launch_select(instance_types, requests, subnet_zones, max_types=60):
    """instance.DefaultProvider.Create's launch-side selection for each (requirements, requests, [type indices])."""
    lib = load()
    arena = abi.Arena()
    desc = arena.catalog_desc(instance_types)
    rq = abi.launch_requests(arena, requests)
    zs = arena.arr(C.c_char_p, [z.encode() for z in subnet_zones])
    out = []
    stride = max_types * max(1, len(subnet_zones))
    for i in range(len(requests)):
        r = abi.LaunchResult()
        types = np.zeros(max_types, dtype=np.uint32)
        ovr = np.zeros(stride, dtype=np.uint32)
        rc = lib.kpo_launch_select(C.byref(desc), C.byref(rq[i]), zs, len(subnet_zones), max_types, C.byref(r),
                                   types.ctypes.data_as(C.POINTER(C.c_uint32)), ovr.ctypes.data_as(C.POINTER(C.c_uint32)))
        if rc != 0:
            raise RuntimeError(f"kpo_launch_select = {rc}")
        out.append(abi.launch_result_dict(r, types, ovr, list(subnet_zones)))
    return out


def requirements_compatible(a, b, allow_wellknown=True):
    lib = load()
    arena = abi.Arena()
    ra, rb = arena.requirements(a), arena.requirements(b)
    return bool(lib.kpo_requirements_compatible(C.byref(ra), C.byref(rb), 1 if allow_wellknown else 0))


def requirements_intersects(a, b):
    lib = load()
    arena = abi.Arena()
    ra, rb = arena.requirements(a), arena.requirements(b)
    return bool(lib.kpo_requirements_intersects(C.byref(ra), C.byref(rb)))


def instance_type_resolve(opts, info, nodeclass):
    lib = load()
    cap, ovh = abi.ResourceList(), Overhead()
    rc = lib.kpo_instance_type_resolve(C.byref(opts), C.byref(info), C.byref(nodeclass), C.byref(cap), C.byref(ovh))
    assert rc == 0
    return cap, ovh


def simulate_batch(cluster, subsets, multi_node=True):
    """computeConsolidation for each candidate subset (list of node indices). Returns (results, stats)."""
    lib = load()
    arena = abi.Arena()
    cl = abi.build_cluster(arena, cluster)
    offs, flat = abi.subsets_csr(arena, subsets)
    out = (abi.SimResult * max(1, len(subsets)))()
    st = abi.SolveStats()
    rc = lib.kpo_simulate_batch(C.byref(cl), offs, flat, len(subsets), 1 if multi_node else 0, out, C.byref(st))
    if rc != 0:
        raise RuntimeError(f"kpo_simulate_batch = {rc}")
    return [sim_dict(out[i]) for i in range(len(subsets))], st


def sim_dict(r):
    return {"decision": r.decision, "nodepool": r.replacement_nodepool, "candidate_price": r.candidate_price,
            "replacement_price": r.replacement_price, "savings": r.savings, "n_options": r.n_options,
            "n_pods": r.n_pods}
