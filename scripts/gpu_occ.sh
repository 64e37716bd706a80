#!/bin/bash
# Occupancy variants: default (4 waves/SIMD, spills) vs w3 (phase A / k_render at 3) vs f3 (phase C at 3).
mkdir -p gpurun_out
for lib in libraycast_hip.so libraycast_hip_c512.so libraycast_hip_c2048.so libraycast_hip.so libraycast_hip_c512.so; do
  line=$(RC_HIP_LIB=$lib timeout -k 10 120 python -u bench.py --timed-only --steps 40 2>>gpurun_out/occ_err.log | grep '^{')
  echo "$lib parity: $(echo "$line" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e9,3), "e9 ms", d["ms_per_step"], "resolver", d["roofline"]["kernel_ms"])' 2>/dev/null)"
  line=$(RC_HIP_LIB=$lib timeout -k 10 120 python -u bench.py --timed-only --steps 40 --mode fast 2>>gpurun_out/occ_err.log | grep '^{')
  echo "$lib fast: $(echo "$line" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e9,3), "e9 ms", d["ms_per_step"])' 2>/dev/null)"
  RC_HIP_LIB=$lib SIZE=4096 TAG="lone $lib" timeout -k 10 120 python -u scripts/lone.py
done
