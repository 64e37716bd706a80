#!/bin/bash
# A/B: frames-in-flight throughput of two library builds, interleaved.
mkdir -p gpurun_out
for lib in libraycast_hip.so libraycast_hip_prev.so libraycast_hip.so libraycast_hip_prev.so libraycast_hip.so libraycast_hip_prev.so; do
  line=$(RC_HIP_LIB=$lib timeout -k 10 120 python -u bench.py --timed-only --steps 40 2>>gpurun_out/ab_err.log | grep '^{')
  echo "$lib: $(echo "$line" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e9,3), "e9 ms", d["ms_per_step"], "resolver", d["roofline"]["kernel_ms"])' 2>/dev/null)"
done
