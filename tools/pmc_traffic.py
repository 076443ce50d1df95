#!/usr/bin/env python3
"""HBM traffic per launch of each bench leg's dominant kernel, from rocprofv3 --pmc passes of tools/prof_leg.py (one
leg per program run, one counter per pass, as the MI355X guide prescribes). Keyed by LEG, so two variants of one
kernel (the price-row and the compact feasibility launches: same kernel, same grid) never share a figure.

Units: rocprofv3 reports kilobytes (1024 B). gfx950 correction (guide, HBM section): FETCH_SIZE counts half the bytes
of wide coalesced reads -> doubled; WRITE_SIZE is exact for streaming stores.

usage: pmc_traffic.py <pmc dir> [out.json]
  <pmc dir>/<leg>_fetch/**/counter_collection.csv and <pmc dir>/<leg>_write/**/counter_collection.csv for every leg"""
import collections
import csv
import glob
import json
import os
import sys

# leg -> (the kernel the bench line's roofline names, its Kernel_Name pattern)
LEGS = {"solve2": ("solve_kernel", "solve_kernel<4, false, false>"),
        "feas_rows": ("feasibility_quad_kernel<7>", "feasibility_quad_kernel<7>"),
        "feas_compact": ("feasibility_quad_kernel<8>", "feasibility_quad_kernel<8>"),
        "sweep": ("sim_kernel", "sim_kernel<"),
        "general": ("solve_kernel<4,*,true>", ", true>(SolveArgs")}


def per_launch(files, counter, pat):
    """(launches, mean counter value per launch) over the dispatches of kernels matching pat."""
    acc = collections.defaultdict(float)
    for f in files:
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter and pat in r["Kernel_Name"]:
                acc[(f, r.get("Dispatch_Id") or r.get("Correlation_Id"))] += float(r["Counter_Value"])
    n = len(acc)
    return n, (sum(acc.values()) / n if n else 0.0)


def main():
    root = sys.argv[1]
    out = {}
    for leg, (kernel, pat) in LEGS.items():
        ff = glob.glob(os.path.join(root, f"{leg}_fetch", "**", "*counter_collection.csv"), recursive=True)
        wf = glob.glob(os.path.join(root, f"{leg}_write", "**", "*counter_collection.csv"), recursive=True)
        if not ff or not wf:
            continue
        nf, f_kb = per_launch(ff, "FETCH_SIZE", pat)
        nw, w_kb = per_launch(wf, "WRITE_SIZE", pat)
        sims = None  # the simulations the profiled run made (consolidation legs: tools/prof_leg.py's JSON line)
        try:
            line = [l for l in open(os.path.join(root, f"{leg}_fetch.log")) if l.startswith("{")][-1]
            sims = json.loads(line).get("subsets")
        except (OSError, IndexError, ValueError):
            pass
        out[leg] = {"kernel": kernel, "kernel_name_match": pat, "launches": [nf, nw],
                    "fetch_size_kb": round(f_kb, 2), "write_size_kb": round(w_kb, 2),
                    "hbm_bytes_per_launch": int(round((2 * f_kb + w_kb) * 1024)),
                    "correction": "2 x FETCH_SIZE + WRITE_SIZE (kB = 1024 B), MI355X_MICROARCH.md HBM section",
                    "source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate runs of tools/prof_leg.py {leg}"}
        if sims:
            out[leg]["sims"] = sims
            out[leg]["hbm_bytes_per_sim"] = round((2 * f_kb + w_kb) * 1024 * nf / sims, 1)
    s = json.dumps(out, indent=1)
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write(s + "\n")
    print(s)


if __name__ == "__main__":
    main()
