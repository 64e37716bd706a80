#!/bin/bash
# Resolver per-segment trace of a lone 4096^2 quadric frame (diagnostic build).
mkdir -p gpurun_out
RC_HIP_LIB=libraycast_hip_stamps.so RC_RESOLVE_TRACE=gpurun_out/trace.txt timeout -k 10 120 python -u scripts/trace_run.py || exit 1
python3 scripts/seg_trace.py gpurun_out/trace.txt | head -40
grep -v "^#" gpurun_out/trace.txt.team | awk '{n[$2]++; c[$2]+=$5} END {for (m in n) print "mode", m, "rounds", n[m], "cycles", c[m]}'
