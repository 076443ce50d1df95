#!/usr/bin/env python3
"""Benchmark: pods scheduled/sec of Scheduler.Solve on MI355X (BASELINE.json metric, config 2).

One step = one Solve of the whole batch on resident inputs (kp_solve_run: restore device state,
solve_kernel, finalize_kernel, copy results back). Compile + upload (kp_solve_prepare) happens once,
untimed, like the catalogue upload it mirrors; its time is reported as prepare_ms.

N > 1 (torchrun, one process per GPU): Solve does not shard (FFD is sequential), so every rank runs an
independent replica of the same batch — weak scaling, no data-path collective. Timing: barrier +
synchronize on both sides, max over ranks (RCCL all-reduce of one float).

cpu_baseline: the oracle (oracle/liboracle.so, single thread, kind "port") on a bounded sample of the
same workload (the config-2 generator with fewer pods), rank 0 at N=1 only.
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
    ap.add_argument("--cpu-sample-pods", type=int, default=10_000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch

    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    import kpamd
    from kpamd import catalog, synth

    lib = kpamd.load_lib()
    cat = catalog.build_catalog(lib)
    prob = synth.config2(cat, n_pods=args.pods, seed=2)
    ctx = kpamd.Context(local)
    plan = kpamd.Scheduler(ctx, prob).prepare()

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    for _ in range(args.warmup):
        plan.run(read=False)
    barrier()
    t0 = time.perf_counter()
    runs = [plan.run(read=False)["stats"] for _ in range(args.steps)]
    barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([elapsed], device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    res = plan.run(read=True)  # one more run for result sanity (not timed)
    placed = int((res["placement"] != -1).sum())
    k_ms = sum(r["solve_kernel_ms"] for r in runs) / len(runs)
    f_ms = sum(r["finalize_kernel_ms"] for r in runs) / len(runs)
    dev_ms = sum(r["device_ms"] for r in runs) / len(runs)
    alg_bytes = sum(r["bytes_algorithmic"] for r in runs) / len(runs)
    prepare_ms = runs[0]["prepare_ms"]
    value = prob.n_pods * world * args.steps / elapsed

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
                        "3 weighted NodePools",
            "pods": prob.n_pods, "instance_types": len(cat), "nodepools": len(prob.nodepools),
            "parallelism": f"replicas x{world} (Solve is sequential FFD; one workgroup per Solve)",
        },
        "device_ms_per_step": round(dev_ms, 3),
        "solve_kernel_ms": round(k_ms, 3),
        "finalize_kernel_ms": round(f_ms, 3),
        "prepare_ms": round(prepare_ms, 1),
        "host_inclusive_pods_per_s": round(prob.n_pods / ((elapsed / args.steps) + prepare_ms / 1e3), 1),
        "nodeclaims": len(res["nodeclaims"]),
        "pods_placed": placed,
        "roofline": {
            "bound": "hbm",
            "kernel": "solve_kernel",
            "achieved": round(alg_bytes / (k_ms / 1e3) / 1e9, 3),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(alg_bytes / (k_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 6),
            "traffic": _traffic(),
            "algorithmic_bytes_per_launch": int(alg_bytes),
            "algorithmic_bytes_per_pod": round(alg_bytes / prob.n_pods, 1),
        },
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = _cpu_baseline(cat, args.cpu_sample_pods)
    if rank == 0:
        print(json.dumps(line), flush=True)
    plan.close()
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()


def _traffic():
    """HBM bytes per solve_kernel launch from the committed rocprofv3 --pmc pass (profiles/), if any."""
    p = os.path.join(REPO, "profiles", "traffic_solve_kernel.json")
    if os.path.exists(p):
        try:
            return json.load(open(p)).get("hbm_bytes_per_launch")
        except Exception:
            return None
    return None


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
