#!/usr/bin/env python3
"""Per-kernel means of rocprofv3 --pmc passes (scripts/pmc_valu.sh) plus derived figures:
  VALU busy   = 4 * SQ_ACTIVE_INST_VALU / (SIMDs * GRBM_GUI_ACTIVE / XCDs)   (quad-cycles -> cycles;
                GRBM_GUI_ACTIVE sums the 8 XCDs' clocks; 4 SIMDs per CU)
  wave state  = SQ_ACTIVE_INST_ANY / SQ_WAIT_ANY / SQ_WAIT_INST_ANY as fractions of SQ_WAVE_CYCLES
  hbm_bytes   = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE counts half of wide reads)
  scripts/pmc_summary.py PMC_DIR OUT.json "config text"
"""
import csv
import json
import os
import sys
from collections import defaultdict

CUS, XCDS = 256, 8


def load(d):
    acc = defaultdict(lambda: defaultdict(list))
    for sub in sorted(os.listdir(d)):
        p = os.path.join(d, sub, "p_counter_collection.csv")
        if not os.path.exists(p):
            continue
        for r in csv.DictReader(open(p)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")
            if "rocclr" in k:
                continue
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in acc.items()}


def main():
    d, out, config = sys.argv[1:4]
    ks = load(d)
    res = {}
    for k, c in ks.items():
        e = {n: round(v) for n, v in sorted(c.items())}
        g = c.get("GRBM_GUI_ACTIVE")
        if g and "SQ_ACTIVE_INST_VALU" in c:
            e["valu_busy"] = round(4 * c["SQ_ACTIVE_INST_VALU"] / (4 * CUS * g / XCDS), 4)
            e["kernel_cycles_per_xcd"] = round(g / XCDS)
        wc = c.get("SQ_WAVE_CYCLES")
        if wc:
            for n in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY"):
                if n in c:
                    e[n.lower().replace("sq_", "frac_")] = round(c[n] / wc, 4)
        if c.get("SQ_THREAD_CYCLES_VALU") and c.get("SQ_ACTIVE_INST_VALU"):   # lanes per VALU op
            e["valu_lane_util"] = round(c["SQ_THREAD_CYCLES_VALU"] / (64 * c["SQ_ACTIVE_INST_VALU"]), 4)
        if c.get("SQ_WAVES") and c.get("SQ_INSTS_VALU"):
            e["valu_insts_per_wave"] = round(c["SQ_INSTS_VALU"] / c["SQ_WAVES"])
        f64 = sum(c.get(f"SQ_INSTS_VALU_{o}_F64", 0) for o in ("ADD", "MUL", "FMA", "TRANS"))
        f32 = sum(c.get(f"SQ_INSTS_VALU_{o}_F32", 0) for o in ("ADD", "MUL", "FMA", "TRANS"))
        if f64 + f32 and c.get("SQ_INSTS_VALU"):
            e["frac_valu_f64_arith"] = round(f64 / c["SQ_INSTS_VALU"], 4)
            e["frac_valu_f32_arith"] = round(f32 / c["SQ_INSTS_VALU"], 4)
        if "FETCH_SIZE" in c or "WRITE_SIZE" in c:
            e["hbm_bytes"] = int(round((2 * c.get("FETCH_SIZE", 0) + c.get("WRITE_SIZE", 0)) * 1024))
        res[k] = e
    json.dump({"config": config, "source": "rocprofv3 --pmc, one pass per counter group "
               "(scripts/pmc_valu.sh); means over dispatches", "kernels": res},
              open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
