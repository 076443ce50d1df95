#!/usr/bin/env python3
"""HBM traffic per launch from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE; one counter per pass as
the MI355X guide prescribes). Units: rocprofv3 reports kilobytes (1024 B). gfx950 correction (guide, HBM
section): FETCH_SIZE counts half the bytes of wide coalesced reads -> doubled; WRITE_SIZE is exact for
streaming stores. usage: pmc_traffic.py <fetch counter_collection.csv> <write counter_collection.csv> [out.json]"""
import collections
import csv
import json
import sys

KERNELS = {"solve_kernel": "solve_kernel<", "feasibility_kernel": "feasibility_kernel(",
           "feasibility_bits_kernel": "feasibility_bits_kernel(", "feasibility_quad_kernel": "feasibility_quad_kernel(",
           "sim_kernel": "sim_kernel<",
           "finalize_kernel": "finalize_kernel("}


def per_kernel(path, counter):
    """{(kernel, grid size): mean counter value per launch} — one kernel launched at several sizes (the
    feasibility leg's 50k-row and 159-row launches) keeps one entry per size."""
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        for k, pat in KERNELS.items():
            if pat in r["Kernel_Name"]:
                acc[(k, int(r["Grid_Size"]))].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main():
    fetch, write = per_kernel(sys.argv[1], "FETCH_SIZE"), per_kernel(sys.argv[2], "WRITE_SIZE")
    out = {}
    for k, grid in sorted(set(fetch) | set(write), key=lambda kg: (kg[0], -kg[1])):
        f_kb, w_kb = fetch.get((k, grid), 0.0), write.get((k, grid), 0.0)
        rec = {"grid_size": grid, "fetch_size_kb": round(f_kb, 2), "write_size_kb": round(w_kb, 2),
               "hbm_bytes_per_launch": int(round((2 * f_kb + w_kb) * 1024)),
               "correction": "2 x FETCH_SIZE + WRITE_SIZE (kB = 1024 B), MI355X_MICROARCH.md HBM section"}
        if k not in out:  # the largest launch of each kernel is its headline entry
            out[k] = dict(rec, other_sizes=[])
        else:
            out[k]["other_sizes"].append(rec)
    s = json.dumps(out, indent=1)
    if len(sys.argv) > 3:
        open(sys.argv[3], "w").write(s + "\n")
    print(s)


if __name__ == "__main__":
    main()
