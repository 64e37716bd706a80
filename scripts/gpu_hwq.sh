#!/bin/bash
# Frames in flight vs the number of hardware queues HIP maps the streams onto.
mkdir -p gpurun_out
for q in 4 8 16 4 8 16; do
  line=$(GPU_MAX_HW_QUEUES=$q timeout -k 10 120 python -u bench.py --timed-only --steps 40 2>>gpurun_out/hwq_err.log | grep '^{')
  echo "hwq $q: $(echo "$line" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e9,3), "e9 ms", d["ms_per_step"], "resolver", d["roofline"]["kernel_ms"])' 2>/dev/null)"
done
