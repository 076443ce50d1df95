#!/usr/bin/env python3
"""Benchmark: pods scheduled/sec of Scheduler.Solve on MI355X (BASELINE.json metric, config 2).

One step = one whole Solve call through the C ABI, kp_solve = kp_solve_prepare + kp_solve_run: compile the batch's
per-Solve half (pod shapes and relaxation levels, existing nodes, topology, the NewQueue sort), upload it, restore
device state, solve_kernel, finalize_kernel, copy the results back. The catalogue half (dictionary, catalogue SoA,
NodeClaimTemplates) is compiled on the first Solve and stays resident in the kp_ctx while the catalogue seqnums
and NodePools are unchanged (R:pkg/providers/instancetype/instancetype.go:225-237 cacheKey); its cold compile time
is reported as catalog_ms. The kp_solve_in (the caller's marshalled pods) is built once, outside the timed region.

N > 1 (torchrun, one process per GPU): Solve does not shard (FFD is sequential), so every rank runs an
independent replica of the same batch — weak scaling, no data-path collective. Timing: barrier +
synchronize on both sides, max over ranks (RCCL all-reduce of one float).

cpu_baseline: the oracle (oracle/liboracle.so, single thread, kind "port") on a bounded sample of the
same workload (the config-2 generator with fewer pods), rank 0 at N=1 only.

Extra legs on the same line (the headline `value` is config 2):
  feasibility   CompatibleAvailableFilter rows x instance types (HBM roofline)
  configs       config 1 (1k pods, kwok pool), config 3 (100k pods, zone + hostname topology spread onto 5k
                existing nodes), config 5 (1M-pod burst, 20 weighted pools with limits, GPU/Neuron pools)
  consolidation config 4 (1M candidate subsets of a 10k-node cluster, sharded over ranks)
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "karpenter-provider-aws_amd"))
sys.path.insert(0, REPO)

METRIC = "pods scheduled/sec (Solve) + consolidation sims/sec, 1–8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--pods", type=int, default=50_000)
    # the headline's CPU baseline at the full config-2 size (50k pods, ~10-25 s of single-threaded oracle time on the
    # GPU box's host): the same machine and the same workload as the device number beside it
    ap.add_argument("--cpu-sample-pods", type=int, default=50_000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cluster-nodes", type=int, default=10_000)
    ap.add_argument("--subsets", type=int, default=1_000_000)
    ap.add_argument("--cpu-sample-sims", type=int, default=16)
    ap.add_argument("--no-consolidation", action="store_true")
    ap.add_argument("--general-nodes", type=int, default=10_000)
    ap.add_argument("--general-subsets", type=int, default=100_000)
    ap.add_argument("--general-max-size", type=int, default=100)
    ap.add_argument("--only-general", action="store_true", help="the topology-cluster consolidation leg alone")
    ap.add_argument("--c3-pods", type=int, default=100_000)
    ap.add_argument("--c5-pods", type=int, default=1_000_000)
    ap.add_argument("--feas-rows", type=int, default=50_000)
    ap.add_argument("--quick", action="store_true", help="config 2 + feasibility only (profiling runs)")
    args = ap.parse_args()
    t_start = time.perf_counter()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch

    # KP_BENCH_BACKEND=gloo rehearses N ranks on a box with fewer GPUs (ranks share GPU local % count); the
    # driver's multi-GPU runs use the default: RCCL ("nccl"), one rank per GPU
    backend = os.environ.get("KP_BENCH_BACKEND", "nccl")
    if backend != "nccl":
        local = local % max(1, torch.cuda.device_count())
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)

    import kpamd
    from kpamd import catalog, synth

    lib = kpamd.load_lib()
    cat = catalog.build_catalog(lib)
    prob = synth.config2(cat, n_pods=args.pods, seed=2)
    ctx = kpamd.Context(local)
    kcomm = None
    if dist is not None and backend == "nccl":  # libkp's RCCL communicator (one rank per GPU): rank 0's unique id
        # shared over torch.distributed; a gloo rehearsal shares GPUs between ranks, which RCCL does not allow
        uid = [kpamd.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        kcomm = kpamd.Comm(ctx, uid[0], world, rank)
    sched = kpamd.Scheduler(ctx, prob)
    sched.solve_in()  # the caller's marshalled batch (Go: the []*v1.Pod it passes to Solve), built once

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    if args.only_general:  # measurement of the general-path leg alone (not the bench contract's line)
        print(json.dumps(_consolidation_general(args, cat, ctx, rank, world, barrier)), flush=True)
        ctx.close()
        return

    def max_over_ranks(x):
        if dist is None:
            return x
        t = torch.tensor([x], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    cold = _solve_step(sched, kcomm)["stats"]  # first Solve on this ctx: compiles the catalogue half (cache miss)
    for _ in range(args.warmup):
        _solve_step(sched, kcomm)
    barrier()
    t0 = time.perf_counter()
    runs = [_solve_step(sched, kcomm)["stats"] for _ in range(args.steps)]
    barrier()
    elapsed = max_over_ranks(time.perf_counter() - t0)

    res = _solve_step(sched, kcomm, read=True)  # one more Solve for result sanity (not timed)
    placed = int((res["placement"] != -1).sum())
    mean = lambda k: sum(r[k] for r in runs) / len(runs)
    k_ms, f_ms, dev_ms = mean("solve_kernel_ms"), mean("finalize_kernel_ms"), mean("device_ms")
    alg_bytes = mean("bytes_algorithmic")
    value = prob.n_pods * world * args.steps / elapsed
    assert all(r["catalog_cached"] == 1 for r in runs), "catalogue half recompiled inside the timed region"

    line = {
        "metric": METRIC,
        "value": round(value, 1),
        "unit": "pods/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int64",
        "data": "synthetic (SURVEY §8d config 2 generator, seed 2; 919-type docs catalogue, splitmix64 spot prices)",
        "config": {
            "workload": "config2: Scheduler.Solve of 50k pending pods (256 deployment shapes: nodeSelector zone, "
                        "node affinity In/Gt, arch NotIn, tolerations) x 919 instance types x 3 AZ x {spot, on-demand}, "
                        "3 weighted NodePools; step = whole kp_solve call (per-Solve compile + upload + kernels + "
                        "result copy-back)",
            "pods": prob.n_pods, "instance_types": len(cat), "nodepools": len(prob.nodepools),
            "parallelism": f"replicas x{world} (Solve is sequential FFD; one workgroup per Solve)" +
                           ("; each Solve's template-options table row-sharded over the ranks + ncclAllGather"
                            if world > 1 else ""),
        },
        "per_solve_prepare_ms": round(mean("prepare_ms"), 3),
        "run_host_ms": round(mean("host_ms"), 3),
        "device_ms_per_step": round(dev_ms, 3),
        "solve_kernel_ms": round(k_ms, 3),
        "finalize_kernel_ms": round(f_ms, 3),
        "catalog_ms": round(cold["catalog_ms"], 3),
        "cold_prepare_ms": round(cold["prepare_ms"], 3),
        "kernel_only_pods_per_s": round(prob.n_pods / (k_ms / 1e3), 1),
        "nodeclaims": len(res["nodeclaims"]),
        "pods_placed": placed,
        "roofline": {
            "bound": "hbm",
            "kernel": "solve_kernel",
            "achieved": round(alg_bytes / (k_ms / 1e3) / 1e9, 3),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(alg_bytes / (k_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 6),
            "traffic": _traffic("solve2"),
            "algorithmic_bytes_per_launch": int(alg_bytes),
            "algorithmic_bytes_per_pod": round(alg_bytes / prob.n_pods, 1),
            "note": "single-workgroup sequential FFD: latency-bound (dependent L2 round trips + barriers per pod)",
            "latency": _latency_roofline(k_ms, prob.n_pods),
        },
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = _cpu_baseline(cat, args.cpu_sample_pods)
        _attach_full_size(line["cpu_baseline"], "config2")
    def progress(msg):  # stderr progress per leg (rank 0): long runs keep writing
        if rank == 0:
            print(f"[bench] {msg} ({time.perf_counter() - t_start:.1f} s)", file=sys.stderr, flush=True)

    progress(f"config2 solve done: {value:.0f} pods/s")
    line["feasibility"] = _feasibility(args, cat, ctx, prob, barrier, max_over_ranks, world)
    progress("feasibility done")
    if not args.quick:
        cfgs = {}
        # config 2 with ReplicaSet bursts (each deployment's pods created within 2 s): 109-pod same-level runs
        cfgs["config2_burst"] = _solve_leg("config2_burst", synth.config2(cat, n_pods=args.pods, seed=2, burst=True), ctx,
                                           barrier, max_over_ranks, world, args.steps, 1, kcomm,
                                           None if (rank or world > 1 or args.no_cpu_baseline) else ("2b", 10_000))
        progress("config2 burst done")
        cfgs["config1"] = _solve_leg("config1", synth.config1(cat, n_pods=1000, seed=1), ctx, barrier,
                                     max_over_ranks, world, args.steps, 1, kcomm,
                                     None if (rank or world > 1 or args.no_cpu_baseline) else ("1", 1000))
        progress("config1 done")
        cfgs["config3"] = _solve_leg("config3", synth.config3(cat, n_pods=args.c3_pods), ctx, barrier,
                                     max_over_ranks, world, 2, 1, kcomm,
                                     None if (rank or world > 1 or args.no_cpu_baseline) else ("3", 3000))
        progress("config3 done")
        cfgs["config5"] = _solve_leg("config5", synth.config5(cat, n_pods=args.c5_pods), ctx, barrier,
                                     max_over_ranks, world, 1, 0, kcomm,
                                     None if (rank or world > 1 or args.no_cpu_baseline) else ("5", 6000))
        line["configs"] = cfgs
    if not args.no_consolidation and not args.quick:
        progress("config5 done")
        line["consolidation"] = _consolidation(args, cat, ctx, dist, rank, world, barrier, kcomm)
        progress("consolidation done")
        line["consolidation_general"] = _consolidation_general(args, cat, ctx, rank, world, barrier)
        progress("general consolidation done")
    if rank == 0:
        print(json.dumps(line), flush=True)
    if kcomm is not None:
        kcomm.close()
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()


def _solve_step(sched, kcomm, read=False):
    """One whole Solve through the C ABI: kp_solve (one process), or with N ranks kp_solve_prepare_comm (the
    template-options table row-sharded over the ranks and all-gathered) + kp_solve_run + destroy."""
    if kcomm is None:
        return sched.solve(read=read)
    plan = sched.prepare(kcomm)
    try:
        return plan.run(read=read)
    finally:
        plan.close()


def _solve_leg(name, prob, ctx, barrier, max_over_ranks, world, steps, warmup, kcomm, cpu):
    """One more BASELINE config as a Solve leg: replicas on every rank, K timed whole kp_solve calls (the catalogue
    half resident after the first). value counts every pod the batch submits; placed_pods_per_s counts the pods
    the Solve placed (existing nodes + new NodeClaims; limits or taints can leave pods unschedulable)."""
    import kpamd
    sched = kpamd.Scheduler(ctx, prob)
    sched.solve_in()
    _solve_step(sched, kcomm)
    for _ in range(warmup):
        _solve_step(sched, kcomm)
    barrier()
    t0 = time.perf_counter()
    runs = [_solve_step(sched, kcomm)["stats"] for _ in range(steps)]
    barrier()
    elapsed = max_over_ranks(time.perf_counter() - t0)
    res = _solve_step(sched, kcomm, read=True)
    k_ms = sum(r["solve_kernel_ms"] for r in runs) / len(runs)
    placed = int((res["placement"] != -1).sum())
    out = {"value": round(prob.n_pods * world * steps / elapsed, 1), "unit": "pods/s", "pods": prob.n_pods,
           "placed_pods_per_s": round(placed * world * steps / elapsed, 1), "pods_placed": placed,
           "steps": steps, "ms_per_step": round(elapsed / steps * 1e3, 2), "solve_kernel_ms": round(k_ms, 2),
           "per_solve_prepare_ms": round(sum(r["prepare_ms"] for r in runs) / len(runs), 2),
           "nodeclaims": len(res["nodeclaims"]),
           "pods_on_existing": int((res["placement"] <= -2).sum()),
           "pods_unschedulable": int((res["placement"] == -1).sum()),
           "workload": prob.name}
    if cpu is not None:
        out["cpu_baseline"] = _cpu_baseline_cfg(cpu[0], cpu[1])
        _attach_full_size(out["cpu_baseline"], {"3": "config3", "5": "config5"}.get(cpu[0]), prob.n_pods)
    return out


def _attach_full_size(cb, name, n_pods=None):
    """The oracle timed on the whole config (tools/cpu_fullsize.py -> profiles/r05/cpu_fullsize.json, committed: the
    full-size runs take minutes to an hour, too long for the bench), beside the bounded sample timed live. The
    sample's rate overstates the CPU where per-pod work grows with the Solve (more NodeClaims to scan)."""
    if not name:
        return
    try:
        rec = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "r05",
                                          "cpu_fullsize.json"))).get(name)
    except (OSError, ValueError):
        rec = None
    if rec and (n_pods is None or rec["pods"] == n_pods):
        cb["full_size"] = {"value": rec["pods_per_s"], "unit": "pods/s", "pods": rec["pods"], "seconds": rec["seconds"],
                           "cores": rec["threads"], "kind": "port",
                           "machine": f"{rec['cpu']} ({rec['host']}): this build's container, not the GPU box"}


def _cpu_baseline_cfg(cfg, n):
    """Oracle Solve, single thread, on a bounded sample of the same generator."""
    from kpamd import catalog, synth
    import kpamd
    from oracle import pyoracle
    cat = catalog.build_catalog(kpamd.load_lib())
    prob = {"1": lambda: synth.config1(cat, n_pods=n, seed=1),
            "2b": lambda: synth.config2(cat, n_pods=n, seed=2, burst=True),
            "3": lambda: synth.config3(cat, n_pods=n, n_deployments=max(1, n // 50), n_existing=max(1, n // 20)),
            "5": lambda: synth.config5(cat, n_pods=n)}[cfg]()
    t0 = time.perf_counter()
    pyoracle.solve(prob)
    dt = time.perf_counter() - t0
    return {"value": round(n / dt, 1), "unit": "pods/s", "cores": 1, "kind": "port",
            "sample": f"{prob.name}: same generator at {n} pods, oracle Solve single-threaded, {dt:.1f} s"}


L2_BYTES_PER_PAIR = 208  # SURVEY §8d type row (64 B value ids + 96 B allocatable + 48 B offerings), L2/MALL-served
ROW_BYTES = 880 + 96     # one compiled requirement row (KReqs) + its requests, read once per row


def _feas_kernel_name(T, prices=True):
    """The bitset filter kernel kp_filter_run launches for a catalogue of T types (csrc launch_feasibility): the quad
    kernel with seven eval waves and a price-row copy wave, or all eight evaluating without price rows."""
    return ("feasibility_quad_kernel<7>" if prices else "feasibility_quad_kernel<8>") if T <= 1024 else \
        "feasibility_bits_kernel"


def _feasibility(args, cat, ctx, prob, barrier, max_over_ranks, world, steps=10):
    """CompatibleAvailableFilter (R:pkg/providers/instance/filter/filter.go:39-64) batched on the device: mask +
    cheapest compatible available offering price per (row, type), rows resident in HBM. Two row sets, both without
    duplicates (SURVEY §8d unit = one (pod shape, type) pair):
      shapes   config 2's distinct NewPodRequirements rows (256 deployment shapes: what one Solve batch needs)
      distinct 50k pairwise-distinct rows (a 50k-deployment cluster's requirement mixes): the HBM roofline leg"""
    import kpamd
    from kpamd import synth
    catalog_h = kpamd.Catalog(ctx, cat)
    rows_c2 = list({(tuple((k, o, tuple(v)) for k, o, v in r), tuple(sorted(q.items()))): (r, q)
                    for r, q in kpamd.pod_queries(prob)}.values())
    legs = {}
    for name, queries in (("shapes", rows_c2), ("distinct", synth.distinct_queries(cat, args.feas_rows))):
        fp = kpamd.FilterPlan(ctx, catalog_h, queries, cheapest=True)
        fp.run()
        barrier()
        t0 = time.perf_counter()
        st = [fp.run() for _ in range(steps)]
        barrier()
        elapsed = max_over_ranks(time.perf_counter() - t0)
        fp.close()
        k_ms = sum(x["device_ms"] for x in st) / steps
        rows, T = len(queries), len(cat)
        pairs = rows * T
        # compulsory HBM bytes: every row read once, every output written once (the 0.2 MB catalogue is resident)
        alg = rows * (ROW_BYTES + 8 * T + 8 * ((T + 63) // 64))
        ach = alg / (k_ms / 1e3) / 1e9
        legs[name] = {"value": round(pairs * world * steps / elapsed, 1), "unit": "pairs/s", "rows": rows,
                      "instance_types": T, "kernel_ms": round(k_ms, 4),
                      "roofline": {"bound": "hbm", "kernel": _feas_kernel_name(T), "achieved": round(ach, 1),
                                   "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
                                   "traffic": _traffic("feas_rows") if name == "distinct" else None,
                                   "algorithmic_bytes_per_launch": alg,
                                   "bytes_per_row": ROW_BYTES + 8 * T + 8 * ((T + 63) // 64),
                                   "l2_effective_GBs": round(pairs * L2_BYTES_PER_PAIR / (k_ms / 1e3) / 1e9, 1)}}
        if name == "distinct":  # the compact result (KP_FILTER_COMPACT): mask + the row's offering classes, no price rows
            fc = kpamd.FilterPlan(ctx, catalog_h, queries, cheapest="compact")
            fc.run_compact(read=False)
            barrier()
            t0 = time.perf_counter()
            stc = [fc.run_compact(read=False) for _ in range(steps)]
            barrier()
            el_c = max_over_ranks(time.perf_counter() - t0)
            fc.close()
            kc_ms = sum(x["device_ms"] for x in stc) / steps
            alg_c = rows * (ROW_BYTES + 8 * ((T + 63) // 64) + 8)
            ach_c = alg_c / (kc_ms / 1e3) / 1e9
            legs[name]["compact"] = {
                "value": round(pairs * world * steps / el_c, 1), "unit": "pairs/s", "kernel_ms": round(kc_ms, 4),
                "roofline": {"bound": "hbm", "kernel": _feas_kernel_name(T, prices=False), "achieved": round(ach_c, 1),
                             "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach_c / HBM_PEAK_GBS, 4),
                             "traffic": _traffic("feas_compact"),
                             "algorithmic_bytes_per_launch": alg_c,
                             "bytes_per_row": ROW_BYTES + 8 * ((T + 63) // 64) + 8},
                "note": "no cheapest-price rows: each row's compatible offering classes (8 B) index the resident "
                        "[classes][types] price table; the evaluation itself, instruction-bound, sets this time"}
    catalog_h.close()
    out = {"metric": "pod-shape x instance-type feasibility pairs/s"}
    out.update(legs["distinct"])
    out["workload"] = f"{legs['distinct']['rows']} distinct requirement rows x {len(cat)} types"
    out["config2_shapes"] = legs["shapes"]
    return out


CHUNK = 1 << 16  # subsets per generation chunk (1M subsets: 16 chunks, contiguous chunk ranges per rank)


def _consolidation(args, cat, ctx, dist, rank, world, barrier, kcomm):
    """Config 4: multi-node consolidation on a 10k-node cluster packed near capacity (delete, replace and no-op
    decisions all occur). Timed, per rank:
      sweep     this rank's contiguous chunk range of the 1M random candidate subsets (2..100 candidates, fixed seed
                per chunk, so the set does not depend on N) through kp_consolidate_argmin: simulation, device argmax,
                and one RCCL all-gather of the ranks' records inside libkp (comm NULL at N=1)
      firstN    rank 0: every prefix firstNConsolidationOption can probe (candidates[0:mid+1], mid = 1..100),
                simulated in one batch, then the binary search replayed (MultiNodeConsolidation's command)
    value = all ranks' subsets / the slowest rank's time."""
    import numpy as np
    import torch
    import kpamd
    from kpamd import disruption, synth

    t0 = time.perf_counter()
    cl = synth.config4(cat, n_nodes=args.cluster_nodes, seed=4)
    cands = np.asarray(cl.candidates, dtype=np.uint32)
    n_chunks = (args.subsets + CHUNK - 1) // CHUNK
    lo, hi = disruption.shard(n_chunks, rank, world)  # contiguous chunk range: balanced for N in 1, 2, 4, 8
    # this rank's chunks concatenated into ONE launch
    sw_offs, sw_nodes, base_index = disruption.sweep_subsets(cands, args.subsets, lo, hi)
    mids = disruption.MultiNodeConsolidation.search_prefixes(len(cands))
    pre = [cands[:m + 1] for m in mids]
    pre_offs = np.zeros(len(pre) + 1, dtype=np.uint32)
    pre_offs[1:] = np.cumsum([len(p) for p in pre])
    pre_nodes = np.concatenate(pre)
    gen_s = time.perf_counter() - t0
    t0 = time.perf_counter()
    plan = kpamd.ClusterPlan(ctx, cl)
    comm = kcomm  # the RCCL communicator lives in libkp (None at N=1)
    prep_all_s = time.perf_counter() - t0
    prep_s = plan.prepare_times["kp_cluster_prepare_s"]  # the library's snapshot build (the per-pass cost)
    warm = min(len(sw_offs) - 1, 1024)  # warmup (untimed) on the first subsets
    plan.argmin(sw_offs[:warm + 1], sw_nodes, base_index=base_index, comm=comm)
    barrier()
    t0 = time.perf_counter()
    choice, st = disruption.sweep(plan, sw_offs, sw_nodes, base_index=base_index, comm=comm)
    first_n = None
    if rank == 0:
        pres, pst = plan.simulate_csr(pre_offs, pre_nodes)
        hit = disruption.MultiNodeConsolidation.replay(len(cands), dict(zip(mids, [kpamd.sim_dict(r) for r in pres])))
        first_n = None if hit is None else {"candidates": hit[0] + 1, "decision": int(hit[1]["decision"]),
                                            "savings": hit[1]["savings"]}
    barrier()
    elapsed = time.perf_counter() - t0
    elapsed_incl = elapsed + prep_s
    n_done = len(sw_offs) - 1 + (len(pre) if rank == 0 else 0)
    total = n_done
    dev = torch.device("cuda", torch.cuda.current_device())
    if dist is not None:
        te = torch.tensor([elapsed, elapsed_incl], dtype=torch.float64, device=dev)
        dist.all_reduce(te, op=dist.ReduceOp.MAX)
        tot = torch.tensor([float(n_done)], dtype=torch.float64, device=dev)
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
        elapsed, elapsed_incl, total = float(te[0].item()), float(te[1].item()), int(tot.item())
    out = {
        "metric": "consolidation sims/s",
        "value": round(total / elapsed, 1),
        "unit": "sims/s",
        "n_gpus": world,
        "scaling": "strong" if world > 1 else "n/a",
        "workload": f"config4: computeConsolidation of {total} candidate subsets ({args.subsets} random subsets of "
                    f"2..100 candidates + {len(pre)} firstNConsolidationOption prefixes) on a {args.cluster_nodes}-node "
                    f"cluster packed near capacity ({len(cl.pod_shape)} pods), 2 NodePools, 919 types; subsets sharded "
                    f"by chunk over ranks, best decision by kp_consolidate_argmin (device argmax + RCCL all-gather)",
        # the disruption controller rebuilds its snapshot every pass: the rate with kp_cluster_prepare inside
        "sims_per_s_incl_prepare": round(total / elapsed_incl, 1),
        "elapsed_incl_prepare_s": round(elapsed_incl, 4),
        "elapsed_s": round(elapsed, 4),
        "sim_kernel_ms_rank0": round(st["solve_kernel_ms"], 3),
        "pods_rescheduled_rank0": int(st["pops"]),
        "roofline": _sim_roofline("sim_kernel", "sweep", st, len(sw_offs) - 1,
                                  "one launch of this rank's sweep subsets; persistent waves, one subset per wave"),
        "decisions": {"noop": choice["counts"][0], "delete": choice["counts"][1], "replace": choice["counts"][2]},
        "best": {"subset": choice["subset"], "decision": choice["result"]["decision"],
                 "savings": choice["result"]["savings"]},
        "first_n": first_n,
        "prepare_s": round(prep_s, 3),
        "prepare_split_s": {k: round(v, 3) for k, v in plan.prepare_times.items()},
        "sims_per_s_incl_prepare_and_marshal": round(total / (elapsed + prep_all_s), 1),
        "subset_generation_s": round(gen_s, 3),
    }
    if rank == 0 and world == 1:  # sims/s by decision class: the first chunk's subsets regrouped by their decision
        n0 = min(CHUNK, len(sw_offs) - 1)
        _, res0, _ = plan.argmin(sw_offs[:n0 + 1], sw_nodes, read_all=True)
        by = {}
        for cls, name in ((0, "noop"), (1, "delete"), (2, "replace")):
            idx = np.nonzero(res0["decision"] == cls)[0]
            if len(idx) < 64:
                continue
            sub = [sw_nodes[sw_offs[i]:sw_offs[i + 1]] for i in idx]
            o = np.zeros(len(sub) + 1, dtype=np.uint32)
            o[1:] = np.cumsum([len(x) for x in sub])
            flat = np.concatenate(sub)
            t1 = time.perf_counter()
            plan.argmin(o, flat)
            torch.cuda.synchronize()
            by[name] = {"subsets": int(len(idx)), "sims_per_s": round(len(idx) / (time.perf_counter() - t1), 1)}
        out["by_decision"] = by
    plan.close()
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = _cpu_baseline_sims(cl, cands, args.cpu_sample_sims)
    return out


def _consolidation_general(args, cat, ctx, rank, world, barrier):
    """Consolidation on a topology-spread cluster (the general simulation path) at config 4's size: a
    10k-node cluster whose every other shape is zone-spread, the 100 firstNConsolidationOption prefixes plus 100k random
    subsets of 2..100 candidates through kp_consolidate_argmin, rank 0 only (each launch of up to 4096 subsets is one
    solve_kernel grid over overlays on the resident superset Solve, two launch slots so the host overlays of one
    overlap the device time of the other; no sharding claimed). Reported with and without kp_cluster_prepare."""
    import numpy as np
    import kpamd
    from kpamd import disruption, synth
    if rank != 0:
        barrier()
        return None
    cl = synth.spread_cluster(cat, args.general_nodes)
    cands = np.asarray(cl.candidates, dtype=np.uint32)
    mids = disruption.MultiNodeConsolidation.search_prefixes(len(cands))
    subs = [list(cands[:m + 1]) for m in mids]
    subs += synth.consolidation_subsets(cl, args.general_subsets, seed=6, max_size=args.general_max_size, prefixes=False)
    offs = np.zeros(len(subs) + 1, dtype=np.uint32)
    offs[1:] = np.cumsum([len(x) for x in subs])
    flat = np.concatenate([np.asarray(x, dtype=np.uint32) for x in subs])
    t0 = time.perf_counter()
    plan = kpamd.ClusterPlan(ctx, cl)
    prep_all_s = time.perf_counter() - t0
    prep_s = plan.prepare_times["kp_cluster_prepare_s"]  # the library's superset compile + upload (per-pass cost)
    prep_split = {k: round(v, 3) for k, v in plan.prepare_times.items()}
    try:
        # warmup (untimed) on the first two launches' worth of subsets: the two launch slots' arenas (~15 MB per
        # simulation here) and pinned buffers are allocated by the first call that needs them and kept by the plan,
        # so the timed pass measures the steady state a disruption loop reusing its plan sees
        warm = min(len(subs), 8192)
        plan.argmin(offs[:warm + 1], flat)
        t0 = time.perf_counter()
        choice, _, st = plan.argmin(offs, flat)
        elapsed = time.perf_counter() - t0
    finally:
        plan.close()
    roof = _sim_roofline("solve_kernel<4,*,true>", "general", st, len(subs),
                         "batched Solves, one workgroup per simulation, launches of up to 4,096 (solve_kernel + "
                         "finalize_kernel time per launch, HIP events)")
    barrier()
    n = len(subs)
    out = {"metric": "consolidation sims/s (general path: topology spread)", "value": round(n / elapsed, 1),
           "unit": "sims/s", "subsets": n, "elapsed_s": round(elapsed, 3), "ms_per_sim": round(elapsed / n * 1e3, 3),
           "sims_per_s_incl_prepare": round(n / (elapsed + prep_s), 1), "prepare_s": round(prep_s, 3),
           "prepare_split_s": prep_split, "sims_per_s_incl_prepare_and_marshal": round(n / (elapsed + prep_all_s), 1),
           "device_ms": round(st["solve_kernel_ms"], 3), "roofline": roof,
           "decisions": {"noop": choice["counts"][0], "delete": choice["counts"][1], "replace": choice["counts"][2]},
           "workload": f"config4 variant: {args.general_nodes} nodes ({len(cl.pod_shape)} pods), every other shape "
                       f"zone-spread (maxSkew 1, DoNotSchedule); {len(mids)} firstNConsolidationOption prefixes + "
                       f"{args.general_subsets} random subsets of 2..{args.general_max_size} candidates; each simulation a whole Solve on the "
                       f"device (host compile + solve_kernel + finalize_kernel), decision on the host"}
    if world == 1 and not args.no_cpu_baseline:
        from oracle import pyoracle
        sample = subs[len(mids):len(mids) + 8]
        t0 = time.perf_counter()
        pyoracle.simulate_batch(cl, sample)
        dt = time.perf_counter() - t0
        out["cpu_baseline"] = {"value": round(len(sample) / dt, 2), "unit": "sims/s", "cores": 1, "kind": "port",
                               "sample": f"8 random subsets of the same cluster, oracle computeConsolidation "
                                         f"single-threaded, {dt:.1f} s"}
    return out


def _sims_worker(arg):
    """One process of the all-threads CPU baseline: the oracle simulates its share of the sample subsets."""
    n_nodes, subs = arg
    import kpamd
    from kpamd import catalog, synth
    from oracle import pyoracle
    cl = synth.config4(catalog.build_catalog(kpamd.load_lib()), n_nodes=n_nodes, seed=4)
    t0 = time.perf_counter()
    pyoracle.simulate_batch(cl, subs)
    return time.perf_counter() - t0


def _cpu_baseline_sims(cl, cands, n, procs=16):
    """computeConsolidation on the CPU oracle: one thread over n subsets of chunk 0, and `procs` processes (the box's
    CPU share; sims parallelize per subset) over procs * n subsets; rate = subsets / the slowest process's time."""
    import multiprocessing as mp
    from kpamd import disruption
    from oracle import pyoracle

    offs, pos = disruption.random_subsets_csr(len(cands), n * procs, seed=1000)
    subs = [[int(x) for x in cands[pos[offs[i]:offs[i + 1]]]] for i in range(n * procs)]
    t0 = time.perf_counter()
    pyoracle.simulate_batch(cl, subs[:n])
    dt = time.perf_counter() - t0
    out = {"value": round(n / dt, 3), "unit": "sims/s", "cores": 1, "kind": "port",
           "sample": f"first {n} random subsets of chunk 0 on the same cluster, oracle computeConsolidation "
                     f"single-threaded, {dt:.1f} s"}
    try:
        with mp.get_context("spawn").Pool(procs) as pool:
            times = pool.map(_sims_worker, [(len(cl.nodes), subs[i::procs]) for i in range(procs)])
        out["all_threads"] = {"value": round(len(subs) / max(times), 3), "unit": "sims/s", "cores": procs,
                              "sample": f"{len(subs)} subsets over {procs} oracle processes (max {max(times):.1f} s)"}
    except Exception as e:  # the single-thread figure stands on its own
        out["all_threads"] = {"error": str(e)[:200]}
    return out


CLOCK_GHZ = 2.4  # MI355X peak engine clock (MI355X_MICROARCH.md chip table)


def _latency_roofline(kernel_ms, pods):
    """The Solve kernel's own bound: one wave issues the whole first-fit loop, so its floor is the issue time of the
    instructions it executes per pod (SQ_ACTIVE_INST_ANY: cycles the waves were issuing; SQ counters from a separate
    rocprofv3 --pmc pass of the same build, tools/pmc_sq.sh -> profiles/latency.json). frac = floor / measured."""
    p = os.path.join(REPO, "profiles", "latency.json")
    if not os.path.exists(p):
        return None
    try:
        lat = json.load(open(p))
        cyc = kernel_ms * 1e-3 * CLOCK_GHZ * 1e9 / pods
        floor = float(lat["issue_cycles_per_pod"])
        return {"cycles_per_pod": round(cyc, 1), "issue_floor_cycles": round(floor, 1), "frac": round(floor / cyc, 4),
                "instructions_per_pod": lat.get("instructions_per_pod"), "source": lat.get("source")}
    except Exception:
        return None


def _traffic(leg):
    """HBM bytes per launch of the leg's kernel from the committed rocprofv3 --pmc passes of tools/prof_leg.py <leg>
    (profiles/traffic.json, written by tools/pmc_traffic.py: one figure per leg, never shared between two variants of
    one kernel), if any."""
    p = os.path.join(REPO, "profiles", "traffic.json")
    if os.path.exists(p):
        try:
            return json.load(open(p)).get(leg, {}).get("hbm_bytes_per_launch")
        except Exception:
            return None
    return None


def _traffic_per_sim(leg):
    p = os.path.join(REPO, "profiles", "traffic.json")
    try:
        return json.load(open(p)).get(leg, {}).get("hbm_bytes_per_sim")
    except Exception:
        return None


def _sim_roofline(kernel, leg, st, n_sims, note):
    """Consolidation legs (SURVEY §8d "Consolidation sim": unit = one subset simulation, B = the bytes its Solve reads
    and writes, counted inside the kernel by the same model as the Solve's): in-kernel algorithmic bytes over the
    kernel's HIP-event time. traffic is per launch of the profiled leg (tools/prof_leg.py), alg_bytes here per launch
    of this run, so compare traffic with algorithmic_bytes_per_sim x the profiled leg's sims per launch."""
    ms = st["solve_kernel_ms"]
    b = float(st["bytes_algorithmic"])
    if ms <= 0 or n_sims <= 0:
        return None
    launches = int(st["phase_cycles"][2]) if leg == "general" else 1  # general path: batched launches of this run
    launches = max(1, launches)
    ach = b / (ms / 1e3) / 1e9
    tps = _traffic_per_sim(leg)
    return {"bound": "hbm", "kernel": kernel, "achieved": round(ach, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(ach / HBM_PEAK_GBS, 6),
            # per launch of this run: the profiled leg's HBM bytes per simulation x this run's simulations per launch
            "traffic": None if tps is None else int(tps * n_sims / launches),
            "traffic_per_sim": tps, "traffic_leg": f"tools/prof_leg.py {leg}",
            "algorithmic_bytes_per_launch": int(b / launches), "algorithmic_bytes_per_sim": round(b / n_sims, 1),
            "launches": launches, "kernel_ms_per_launch": round(ms / launches, 3), "sims": n_sims, "note": note}


def _cpu_baseline(cat, n_pods):
    from kpamd import synth
    from oracle import pyoracle

    prob = synth.config2(cat, n_pods=n_pods, seed=2)
    t0 = time.perf_counter()
    pyoracle.solve(prob)
    dt = time.perf_counter() - t0
    cpu = "unknown"
    try:
        for l in open("/proc/cpuinfo"):
            if l.startswith("model name"):
                cpu = l.split(":", 1)[1].strip()
                break
    except Exception:
        pass
    return {"value": round(n_pods / dt, 1), "unit": "pods/s", "cores": 1, "kind": "port",
            "sample": f"config2 generator with {n_pods} pods (same shapes/seed), oracle Solve single-threaded, "
                      f"{dt:.1f} s on {cpu}"}


if __name__ == "__main__":
    main()
