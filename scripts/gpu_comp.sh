#!/bin/bash
# Compaction stream A/B (frames in flight), 4096^2 and 8192^2, interleaved; then the frames-in-flight tests.
mkdir -p gpurun_out
for sz in 4096 8192; do
for cs in 1 0 1 0 1 0; do
  line=$(timeout -k 10 120 python -u bench.py --timed-only --size $sz --steps 30 --tune comp_stream=$cs 2>>gpurun_out/comp_err.log | grep '^{')
  echo "size $sz comp_stream $cs: $(echo "$line" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e9,3), "e9 ms", d["ms_per_step"], "resolver", d["roofline"]["kernel_ms"])' 2>/dev/null)"
done; done
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread -k "frames_in_flight or bench_sequence or phantom" > gpurun_out/pt.log 2>&1; tail -1 gpurun_out/pt.log
