#!/bin/bash
# Coalesced carry-in publication: parity suite subset, lone/bench timing, k_resolve WRITE_SIZE.
set -o pipefail
mkdir -p gpurun_out/pmc_cin
export TMPDIR=/tmp
bash scripts/gpu_perf.sh || exit 1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_cin/write -o p -- python -u scripts/lone.py > gpurun_out/pmc_cin/write.log 2>&1 || { echo "pmc failed"; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_cin/fetch -o p -- python -u scripts/lone.py > gpurun_out/pmc_cin/fetch.log 2>&1 || { echo "pmc failed"; exit 1; }
python3 - <<'PY'
import csv, collections
for pas in ("write", "fetch"):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f"gpurun_out/pmc_cin/{pas}/p_counter_collection.csv")):
        acc[r["Kernel_Name"].split("(")[0][:30]].append(float(r["Counter_Value"]))
    for k, v in acc.items():
        if "resolve" in k or "side" in k or "phase_a" in k:
            print(pas, k, round(sum(v) / len(v) * 1024 / 1e6, 1), "MB per launch")
PY
