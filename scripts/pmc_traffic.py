#!/usr/bin/env python3
"""Per-kernel HBM traffic from two rocprofv3 counter-collection passes (FETCH_SIZE and
WRITE_SIZE, collected separately as MI355X_MICROARCH.md prescribes):
hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 per dispatch, FETCH doubled because gfx950's
FETCH_SIZE counts half of wide streaming reads.  Mean over each kernel's dispatches.

  scripts/pmc_traffic.py FETCH.csv WRITE.csv OUT.json "config text"
"""
import csv
import json
import sys
from collections import defaultdict


def kname(raw):
    n = raw.split("(")[0]
    return n[5:] if n.startswith("void ") else n


def means(path, counter):
    acc = defaultdict(list)
    with open(path) as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] == counter:
                acc[kname(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main():
    fetch, write, out, config = sys.argv[1:5]
    f, w = means(fetch, "FETCH_SIZE"), means(write, "WRITE_SIZE")
    kernels = {}
    for k in sorted(set(f) | set(w)):
        d = {"FETCH_SIZE_KB": round(f.get(k, 0.0), 3), "WRITE_SIZE_KB": round(w.get(k, 0.0), 3)}
        d["hbm_bytes"] = int(round((2 * f.get(k, 0.0) + w.get(k, 0.0)) * 1024))
        kernels[k] = d
    with open(out, "w") as fo:
        json.dump({"config": config,
                   "source": "rocprofv3 --pmc FETCH_SIZE --kernel-trace / --pmc WRITE_SIZE "
                             "--kernel-trace, separate passes (scripts/pmc_traffic.py)",
                   "units": "FETCH_SIZE/WRITE_SIZE raw in KB per dispatch (mean over "
                            "dispatches); hbm_bytes = 2*FETCH + WRITE per MI355X_MICROARCH.md "
                            "(gfx950 FETCH_SIZE counts half of wide streaming reads)",
                   "kernels": kernels}, fo, indent=1)


if __name__ == "__main__":
    main()
